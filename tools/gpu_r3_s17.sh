# side-stream LSTM weight-gradient workgroup cap A/B (AVC_LSTM_WG_TARGET), interleaved, 3 reps
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r3s17}
mkdir -p $OUT
for r in 1 2 3; do
  for t in 0 192 128 64; do
    echo -n "target $t rep $r: " >> $OUT/cap_ab.log
    AVC_LSTM_WG_TARGET=$t timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> $OUT/cap_ab.log || exit 1
  done
done
cat $OUT/cap_ab.log
