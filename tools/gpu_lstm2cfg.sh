# Wavefront forward configurations (AVC_LSTM2_CFG): tests, timelines and bench lines -> gpurun_out/$1
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-lstm2cfg}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
(cd $R && timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "lstm2" -x -q --timeout 120 \
    --timeout-method thread > $OUT/pytest.log 2>&1) || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for cfg in ${CFGS:-20 10 21}; do
  AVC_LSTM2_CFG=$cfg timeout -k 10 150 python $R/tools/lstm_trace.py > $OUT/trace_$cfg.log 2>&1 || { cat $OUT/trace_$cfg.log; exit 1; }
  echo "CFG=$cfg"; grep -E "lstm2" $OUT/trace_$cfg.log
  AVC_LSTM2_CFG=$cfg timeout -k 10 200 python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err || { tail $OUT/bench_$cfg.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_$cfg.json')); print('CFG=$cfg', d['ms_per_step'], d['value'])"
done
