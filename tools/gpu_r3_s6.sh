# LSTM backward DIRECT form: parity (incl. under load), timeline A/B, bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r3s6}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "persistent_backward" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 120 python -u tools/lstm_trace.py > $OUT/trace_direct.log 2>&1 || exit 1
AVC_LSTM_BWD_DIRECT=0 timeout -k 10 120 python -u tools/lstm_trace.py > $OUT/trace_lds.log 2>&1 || exit 1
for r in 1 2; do
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | cut -c1-200 >> $OUT/bench_direct.log || exit 1
AVC_LSTM_BWD_DIRECT=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | cut -c1-200 >> $OUT/bench_lds.log || exit 1
done
for f in 1 0; do
  echo "== AVC_CONV0_FOLD=$f" >> $OUT/margin.log
  AVC_CONV0_FOLD=$f timeout -k 10 120 python -u tools/bf16_margin.py >> $OUT/margin.log 2>&1 || exit 1
  AVC_CONV0_FOLD=$f timeout -k 10 200 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_variants.py -k "gpu_variant_step and Adjust" >> $OUT/margin.log 2>&1
done
for v in "AVC_GRAPH_SERIAL=1 AVC_GRAPH_SEGMENTS=1 AVC_GRAPH_SKIP_SIDE=1" "AVC_GRAPH_SPLIT=0"; do
  echo "== $v" >> $OUT/graph_check.log
  env $v timeout -k 10 150 python -u tools/graph_check.py 3 >> $OUT/graph_check.log 2>&1 || exit 1
done
