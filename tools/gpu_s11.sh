# kernel + model tests, then one kernel-trace profile of the bench step (loss-block timing)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/s11; mkdir -p $OUT
(cd $R && timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_variants.py -m gpu -x -q \
   --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1) || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p -o run -- \
    python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing > $OUT/p.log 2>&1 || exit 1
grep -h "vc_loss\|adam_kernel" $OUT/p/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
