# granule vs flag hand-off of the persistent recurrences: parity (both forms), step timeline, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/gran; mkdir -p $O
AVC_LSTM_GRAN=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_fault.py -m gpu -k "lstm or persist or fault" > $O/t_gran.log 2>&1 || { tail -30 $O/t_gran.log; exit 1; }
tail -2 $O/t_gran.log
for m in 0 3; do
  AVC_LSTM_GRAN=$m timeout -k 10 120 python -u tools/lstm_trace.py > $O/trace_$m.log 2>&1 || exit 1
  cat $O/trace_$m.log | grep -v amdgpu.ids
done
for m in 0 1 2 3 0 3; do
  AVC_LSTM_GRAN=$m timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$m.json 2>$O/bench_$m.err || exit 1
  python -c "import json,sys; d=json.load(open('$O/bench_$m.json')); print('GRAN=$m', d['ms_per_step'], d['value'])"
done
