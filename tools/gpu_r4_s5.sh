# round 4: full GPU suite (+B=64 oracle bars), C2 / C4 / C5 benches, host enqueue, graph queues, LSTM payload ablation
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 900 --timeout-method thread -rA \
    > $OUT/pytest_gpu.log 2>&1 || { grep -a "vs oracle" $OUT/pytest_gpu.log; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
grep -a "vs oracle" $OUT/pytest_gpu.log
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/c2.$rep.json 2>/dev/null || exit 1
  timeout -k 10 200 python -u bench.py --model MetaConv --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c4.$rep.json 2>/dev/null || exit 1
done
timeout -k 10 200 python -u bench.py --disc --steps 20 --warmup 3 --no-cpu-baseline > $OUT/c5.json 2>/dev/null || exit 1
timeout -k 10 200 python -u tools/host_time.py --steps 30 > $OUT/host_time.txt 2>&1 || exit 1
tail -2 $OUT/host_time.txt
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --graph > $OUT/graph_q0.json 2>$OUT/graph_q0.err || exit 1
for q in 2 4; do
  DEBUG_HIP_FORCE_GRAPH_QUEUES=$q timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --graph \
      > $OUT/graph_q$q.json 2>$OUT/graph_q$q.err || exit 1
done
timeout -k 10 200 python -u tools/lstm_trace.py > $OUT/lstm_trace.txt 2>&1 || exit 1
AVC_LSTM_BWD_ABL=1 timeout -k 10 200 python -u tools/lstm_trace.py > $OUT/lstm_trace_abl.txt 2>&1 || exit 1
grep -a "bwd" $OUT/lstm_trace.txt $OUT/lstm_trace_abl.txt
grep -o '"ms_per_step": [0-9.]*' $OUT/*.json
timeout -k 10 200 python -u tools/blas_probe2.py > $OUT/blas_probe2.txt 2>&1 || exit 1
cat $OUT/blas_probe2.txt
