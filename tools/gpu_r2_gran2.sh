# granule sweep back-off (AVC_LSTM_NAP) on the step timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/gran2; mkdir -p $O
for n in 0 1 2 4 8; do
  echo "== NAP=$n"
  AVC_LSTM_GRAN=3 AVC_LSTM_NAP=$n timeout -k 10 120 python -u tools/lstm_trace.py > $O/trace_$n.log 2>&1 || exit 1
  grep "events" $O/trace_$n.log
done
