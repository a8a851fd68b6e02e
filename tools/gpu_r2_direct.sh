# backward direct-fragment form (AVC_LSTM_DIRECT) + default granule lstm1 forward: parity, timeline, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/direct; mkdir -p $O
AVC_LSTM_DIRECT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_fault.py -m gpu -k "lstm or persist or fault" > $O/t_direct.log 2>&1 || { tail -30 $O/t_direct.log; exit 1; }
tail -1 $O/t_direct.log
for m in 0 1; do
  AVC_LSTM_DIRECT=$m timeout -k 10 120 python -u tools/lstm_trace.py > $O/trace_$m.log 2>&1 || exit 1
  grep -v amdgpu.ids $O/trace_$m.log
done
for m in 0 1 0 1; do
  AVC_LSTM_DIRECT=$m timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$m.json 2>$O/bench_$m.err || exit 1
  python -c "import json,sys; d=json.load(open('$O/bench_$m.json')); print('DIRECT=$m', d['ms_per_step'], d['value'])"
done
