# Partial-sum backward A/B: kernel tests (both forms), LSTM step timelines and bench lines
# for AVC_LSTM_BWD_PS=1 (default) and =0 on the same box -> gpurun_out/$1
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-ps}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
(cd $R && timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "persistent_backward" -x -q --timeout 120 \
    --timeout-method thread > $OUT/pytest_ps.log 2>&1) || { tail -30 $OUT/pytest_ps.log; exit 1; }
tail -2 $OUT/pytest_ps.log
for f in 1 0 1; do
  AVC_LSTM_BWD_PS=$f timeout -k 10 120 python $R/tools/lstm_trace.py > $OUT/trace_$f.log 2>&1 || { cat $OUT/trace_$f.log; exit 1; }
  echo "== PS=$f"; grep -E "bwd" $OUT/trace_$f.log
  AVC_LSTM_BWD_PS=$f timeout -k 10 200 python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_$f.json 2> $OUT/bench_$f.err || { tail $OUT/bench_$f.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_$f.json')); print('PS=$f', d['ms_per_step'], d['value'], d['roofline']['avg_us'])"
done
