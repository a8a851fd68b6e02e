# Round-6 closing pass: full GPU suite, the closing measurements (tools/gpu_close.sh, prefix r6) and the other configs
#   gpurun --timeout 1200 -- bash tools/gpu_r6_close.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r6close}
mkdir -p $R/gpurun_out/$TAG
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1 || { tail -30 gpurun_out/$TAG/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$TAG/gpu_tests.log
bash tools/gpu_close.sh $TAG r6 && bash tools/gpu_configs.sh ${TAG}_configs
