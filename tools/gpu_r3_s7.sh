set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r3s7}
mkdir -p $OUT
for f in 1 0; do
  echo "== AVC_CONV0_FOLD=$f" >> $OUT/margin.log
  AVC_CONV0_FOLD=$f timeout -k 10 120 python -u tools/bf16_margin.py >> $OUT/margin.log 2>&1 || exit 1
done
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -rf -m gpu \
  tests/test_gpu_model.py tests/test_variants.py tests/test_gpu_kernels.py tests/test_gpu_metaformer.py > $OUT/model.log 2>&1; echo "model rc $?" >> $OUT/model.log
tail -4 $OUT/model.log
for v in "AVC_GRAPH_SPLIT=0" "AVC_GRAPH_SERIAL=1 AVC_GRAPH_SEGMENTS=1 AVC_GRAPH_SKIP_SIDE=1"; do
  echo "== $v" >> $OUT/graph_check.log
  env $v timeout -k 10 150 python -u tools/graph_check.py 3 >> $OUT/graph_check.log 2>&1 || exit 1
done
timeout -k 10 200 python -u tools/blas_probe.py > $OUT/blas_probe.log 2>&1 || exit 1
for r in 1 2; do
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | cut -c1-200 >> $OUT/bench_fold.log || exit 1
AVC_CONV0_FOLD=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | cut -c1-200 >> $OUT/bench_nofold.log || exit 1
done
