# round 5: deferred lstm2 weight gradients -- tests, C2 A/B
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r5df}
mkdir -p $O
#timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_replay.py tests/test_gpu_capture.py tests/test_gpu_model.py > $O/t.txt 2>&1
bash tools/ab_replay.sh ${1:-r5df} "AVC_DEFER_LSTM2_WG=2" "AVC_DEFER_LSTM2_WG=0" "AVC_DEFER_LSTM2_WG=1"
