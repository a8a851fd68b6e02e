# round 5: TT split-K reduction without atomics -- tests, C2 A/B
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r5sk}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "tt or split or conv" > $O/t_kernels.txt 2>&1
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_capture.py tests/test_gpu_model.py > $O/t_capture.txt 2>&1
bash tools/ab_replay.sh ${1:-r5sk} "AVC_TT_SPLITK=8" "AVC_TT_SPLITK=8 AVC_CONV_DW_DIRECT=0" "AVC_TT_SPLITK=0"
