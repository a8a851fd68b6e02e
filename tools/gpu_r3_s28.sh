# zero_grad on the side stream: TrainStep tests, host time, bench x3
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r3s28}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_graph.py tests/test_gpu_model.py tests/test_gpu_disc.py tests/test_gpu_fault.py tests/test_gpu_dist.py tests/test_gpu_capture.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python -u tools/host_time.py > $OUT/host_time.log 2>&1 || exit 1
for r in 1 2 3; do timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> $OUT/bench.log || exit 1; done
cat $OUT/host_time.log $OUT/bench.log
