# per-wave flag hand-off (AVC_LSTM_PW): parity, step timeline, interleaved bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/pw; mkdir -p $O
AVC_LSTM_PW=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_fault.py -m gpu -k "lstm or persist or fault" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for m in 0 1; do
  AVC_LSTM_PW=$m timeout -k 10 120 python -u tools/lstm_trace.py > $O/trace_$m.log 2>&1 || exit 1
  echo "PW=$m"; grep -v amdgpu.ids $O/trace_$m.log
done
bash tools/ab.sh "AVC_LSTM_PW=0" "AVC_LSTM_PW=1" 3
