# LSTM backward wave-local staging (AVC_LSTM_BWD_WL) parity + timeline + step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r3s15}
mkdir -p $OUT
AVC_LSTM_BWD_WL=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "persistent_backward" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
AVC_LSTM_BWD_WL=1 timeout -k 10 120 python -u tools/lstm_trace.py > $OUT/trace_wl.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/lstm_trace.py > $OUT/trace_def.log 2>&1 || exit 1
grep "bwd" $OUT/trace_wl.log $OUT/trace_def.log
for r in 1 2; do
timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline 2>/dev/null | cut -c1-200 >> $OUT/bench_def.log || exit 1
AVC_LSTM_BWD_WL=1 timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline 2>/dev/null | cut -c1-200 >> $OUT/bench_wl.log || exit 1
done
grep -o '"ms_per_step": [0-9.]*' $OUT/bench_def.log $OUT/bench_wl.log
