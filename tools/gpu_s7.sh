# kernel tests, then same-box A/B against the _ab_head/ copy
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/s7
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/s7/pytest.log 2>&1 || { tail -40 gpurun_out/s7/pytest.log; exit 1; }
tail -1 gpurun_out/s7/pytest.log
bash tools/ab_head.sh "--steps 30 --warmup 5" "AVC_BNB=0" 2
