# Host-side diagnosis + graph A/B + capture numbers + C4/C5 re-measure.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r3s2}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_capture.py -q -s --timeout 280 --timeout-method thread > $OUT/capture.log 2>&1
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -q --timeout 120 --timeout-method thread -k "weight_gradient_window" > $OUT/halo.log 2>&1 || { tail -20 $OUT/halo.log; exit 1; }
timeout -k 10 200 python -u tools/host_time.py --steps 20 > $OUT/host_time.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/host_profile.py > $OUT/host_profile.log 2>&1 || exit 1
for v in "AVC_GRAPH_SPLIT=0" "AVC_GRAPH_SPLIT=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=4" "AVC_GRAPH_SPLIT=1"; do
  echo "== $v" >> $OUT/graph.log
  env $v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --graph --no-cpu-baseline --no-kernel-timing 2>>$OUT/graph.err | cut -c1-200 >> $OUT/graph.log || exit 1
done
timeout -k 10 300 python -u bench.py --model MetaConv --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_MetaConv.json 2>/dev/null &&
timeout -k 10 300 python -u bench.py --disc --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_disc.json 2>/dev/null || exit 1
