# MLPMixer weight gradients on the side stream (AVC_MIX_SIDE): tests + interleaved C4 / MetaPool A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r3s34}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
timeout -k 10 800 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_metaformer.py tests/test_variants.py tests/test_gpu_model.py tests/test_gpu_capture.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for r in 1 2 3; do
  for f in 1 0; do
    echo -n "C4 mixside $f rep $r: " >> $OUT/ab.log
    AVC_MIX_SIDE=$f timeout -k 10 300 python -u bench.py --model MetaConv --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> $OUT/ab.log || exit 1
  done
done
for f in 1 0; do
  echo -n "MetaPool mixside $f: " >> $OUT/ab.log
  AVC_MIX_SIDE=$f timeout -k 10 300 python -u bench.py --model MetaPool --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> $OUT/ab.log || exit 1
done
cat $OUT/ab.log
