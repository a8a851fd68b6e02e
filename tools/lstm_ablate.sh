set -e
for m in 0 1 2 3; do echo "dbg=$m"; AVC_LSTM_DEBUG=$m timeout -k 10 120 python tools/lstm_bench.py 2>&1 | grep -v amdgpu | head -1; done
