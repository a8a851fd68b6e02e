# Round-3 first pass: whole GPU suite (incl. the op capture), LSTM timeline, bench, kernel
# stats, backward hand-off forms A/B.   gpurun --timeout 1150 -- bash tools/gpu_r3_s1.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3s1}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
(cd $R && timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf \
    > $OUT/pytest_gpu.log 2>&1); rc=$?
tail -5 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 120 python $R/tools/lstm_trace.py > $OUT/lstm_trace.log 2>&1 &&
timeout -k 10 300 python $R/bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err &&
cat $OUT/bench.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1 &&
(cd $R && HS=1024,512 FORMS=0,2,3 timeout -k 10 200 python -u tools/lstm_bwd_forms.py 3 > $OUT/forms.log 2>&1) || exit 1
exit $rc
