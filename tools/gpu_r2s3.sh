# Session-3 batch: lstm2 tests, LSTM timelines, and same-box A/B of the main-stream priority and
# of exclusive-LDS recurrences -> gpurun_out/$1
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r2s3}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
(cd $R && timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "lstm2 or persistent_backward" -x -q --timeout 120 \
    --timeout-method thread > $OUT/pytest.log 2>&1) || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 150 python $R/tools/lstm_trace.py > $OUT/trace.log 2>&1 || { cat $OUT/trace.log; exit 1; }
grep -v amdgpu.ids $OUT/trace.log
bash $R/tools/gpu_envab.sh ${1:-r2s3}/ab "AVC_MAIN_PRIO=0" "AVC_MAIN_PRIO=1" "AVC_LSTM_EXCL=1" "AVC_LSTM2_OFF=1"
