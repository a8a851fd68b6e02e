# Wavefront two-layer forward: kernel + autograd tests, then the step with and without it
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-lstm2}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
(cd $R && timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "lstm2 or persistent_forward" -x -q --timeout 120 \
    --timeout-method thread > $OUT/pytest.log 2>&1) || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for f in 0 1 0; do
  if [ $f = 1 ]; then export AVC_LSTM2_OFF=1; else unset AVC_LSTM2_OFF; fi
  timeout -k 10 200 python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_off$f.json 2> $OUT/bench_off$f.err || { tail $OUT/bench_off$f.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_off$f.json')); print('LSTM2_OFF=$f', d['ms_per_step'], d['value'], d['final_loss'])"
done
unset AVC_LSTM2_OFF
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit 1
head -12 $OUT/prof/run_kernel_stats.csv | cut -c1-160
