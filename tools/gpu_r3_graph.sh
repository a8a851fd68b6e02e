set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_graph.py tests/test_gpu_model.py -k "graph" > gpurun_out/r3u_tests.log 2>&1 || exit 1
O=gpurun_out/r3u.log
echo "eager" >> $O
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing 2>/dev/null | cut -c1-260 >> $O || exit 1
for sg in 4 16 64; do
echo "graph split segments $sg" >> $O
AVC_GRAPH_SEGMENTS=$sg timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --graph --no-cpu-baseline --no-kernel-timing 2>/dev/null | cut -c1-260 >> $O || exit 1
done
