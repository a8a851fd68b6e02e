# round 4: host enqueue vs GPU step (C2) and a cProfile of the step's host side -> gpurun_out/$1
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
timeout -k 10 200 python -u tools/host_time.py --steps 30 > $OUT/host_time.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/host_profile2.py > $OUT/host_profile2.txt 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/c2.json 2>/dev/null || exit 1
cat $OUT/host_time.txt | tail -3
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -x -q -s --timeout 900 --timeout-method thread -k "b64 or loose" \
    > $OUT/b64.log 2>&1 || { tail -30 $OUT/b64.log; exit 1; }
grep -a "vs oracle" $OUT/b64.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "colsum or bias" \
    > $OUT/colsum.log 2>&1 || { tail -30 $OUT/colsum.log; exit 1; }
tail -1 $OUT/colsum.log
timeout -k 10 200 python -u tools/lstm_trace.py > $OUT/lstm_trace.txt 2>&1 || exit 1
AVC_LSTM_BWD_ABL=1 timeout -k 10 200 python -u tools/lstm_trace.py > $OUT/lstm_trace_abl.txt 2>&1 || exit 1
grep -a "bwd" $OUT/lstm_trace.txt $OUT/lstm_trace_abl.txt
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --model MetaConv --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c4.$rep.json 2>/dev/null || exit 1
done
grep -o '"ms_per_step": [0-9.]*' $OUT/*.json
