# BN backward fused finalize tests + A/B, WL backward A/B, weight-gradient cap A/B, disc/C4/C2 profile
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r3s19}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "bn" > $OUT/bn_tests.log 2>&1 || { tail -30 $OUT/bn_tests.log; exit 1; }
tail -2 $OUT/bn_tests.log
for r in 1 2 3; do
  for f in 1 0; do
    echo -n "bnfuse $f rep $r: " >> $OUT/bn_ab.log
    AVC_BN_BWD_FUSE=$f timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> $OUT/bn_ab.log || exit 1
  done
done
cat $OUT/bn_ab.log
bash $R/tools/gpu_r3_s15.sh $T || exit 1
bash $R/tools/gpu_r3_s17.sh $T || exit 1
bash $R/tools/gpu_r3_s14.sh $T || exit 1
