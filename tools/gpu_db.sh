# round 5: wavefront backward with bf16 dG + bias partials (ABI 28) -- tests, isolated timing, C2 A/B
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r5db}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lstm2_bwd.py > $O/t1.txt 2>&1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_capture.py tests/test_gpu_model.py tests/test_gpu_replay.py tests/test_gpu_dist.py > $O/t2.txt 2>&1
timeout -k 10 120 python -u tools/lstm2_bwd_bench.py 10 > $O/bench_tool.txt 2>&1
bash tools/ab_replay.sh ${1:-r5db} "AVC_LSTM2_DB=1" "AVC_LSTM2_DB=0"
