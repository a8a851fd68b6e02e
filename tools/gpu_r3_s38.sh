# BiLSTM forward staging after the barrier: tests, timeline, bench
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r3s38}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_capture.py -k "lstm or model or golden or capture" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 120 python -u tools/lstm_trace.py > $OUT/trace.log 2>&1 || exit 1
grep BiLSTM $OUT/trace.log
for r in 1 2 3; do timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> $OUT/bench.log || exit 1; done
cat $OUT/bench.log
