# conv0 fold: kernel + layer + model parity, capture; graph-split bisect; C2 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r3s5}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_kernels.py -k "fold or weight_gradient_window" > $OUT/fold_kernels.log 2>&1 || { tail -30 $OUT/fold_kernels.log; exit 1; }
timeout -k 10 500 python -u -m pytest -q --timeout 300 --timeout-method thread -rf \
  tests/test_gpu_model.py tests/test_variants.py tests/test_gpu_fold.py tests/test_gpu_disc.py > $OUT/model.log 2>&1; echo "model rc $?" >> $OUT/model.log
tail -3 $OUT/model.log
timeout -k 10 300 python -u -m pytest -q -s --timeout 280 --timeout-method thread tests/test_gpu_capture.py > $OUT/capture.log 2>&1; echo "capture rc $?" >> $OUT/capture.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2>/dev/null || exit 1
AVC_CONV0_FOLD=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_nofold.json 2>/dev/null || exit 1
for v in "AVC_GRAPH_SERIAL=1 AVC_GRAPH_SEGMENTS=1" "AVC_GRAPH_SERIAL=1 AVC_GRAPH_RUNS=1" "AVC_GRAPH_RUNS=1"; do
  echo "== $v" >> $OUT/graph_check.log
  env $v timeout -k 10 150 python -u tools/graph_check.py 3 >> $OUT/graph_check.log 2>&1 || exit 1
done
