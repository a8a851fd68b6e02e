# kernel-trace profiles of the C2 bench: last-block backward finalize (p_bn1) and separate launch (p_bn0)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "bn" > gpurun_out/t_k.log 2>&1 || exit 1
bash tools/gpu_prof.sh p_bn1 || exit 1
AVC_LAST_BLOCK=0 bash tools/gpu_prof.sh p_bn0
