set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "persistent_backward" > gpurun_out/r3a_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/lstm_bwd_forms.py 3 > gpurun_out/r3a_forms.log 2>&1
