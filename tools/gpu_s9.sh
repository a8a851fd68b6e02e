# kernel stats of the bench step with and without the fused BN-backward statistics (AVC_BNB)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/s9; mkdir -p $OUT
(cd $R && timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "bnb or chain or apply" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1) || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  AVC_BNB=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p$v -o run -- \
      python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing > $OUT/p$v.log 2>&1 || exit 1
  grep ms_per_step $OUT/p$v.log | head -1
done
