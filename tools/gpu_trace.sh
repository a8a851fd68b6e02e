# LSTM step timelines (tools/lstm_trace.py) -> gpurun_out/$1/trace.log
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-trace}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 150 python $R/tools/lstm_trace.py > $OUT/trace.log 2>&1; rc=$?; cat $OUT/trace.log; exit $rc
