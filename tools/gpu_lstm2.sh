# Wavefront two-layer forward: kernel + autograd tests, timelines (SB variants), then the step
# with and without it -> gpurun_out/$1
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-lstm2}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
(cd $R && timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "lstm2 or persistent" -x -q --timeout 120 \
    --timeout-method thread > $OUT/pytest.log 2>&1) || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for sb in 2 4; do
  AVC_LSTM2_SB=$sb timeout -k 10 150 python $R/tools/lstm_trace.py > $OUT/trace_sb$sb.log 2>&1 || { cat $OUT/trace_sb$sb.log; exit 1; }
  echo "SB=$sb"; grep -E "lstm2|H=1024 fwd" $OUT/trace_sb$sb.log
done
for f in 0 1 0; do
  if [ $f = 1 ]; then export AVC_LSTM2_OFF=1; else unset AVC_LSTM2_OFF; fi
  timeout -k 10 200 python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_off$f.json 2> $OUT/bench_off$f.err || { tail $OUT/bench_off$f.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_off$f.json')); print('LSTM2_OFF=$f', d['ms_per_step'], d['value'], d['final_loss'])"
done
