set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/golden_margin.py > gpurun_out/margin.log 2>&1 || exit 1
AVC_FOLD=0 timeout -k 10 200 python -u tools/golden_margin.py >> gpurun_out/margin.log 2>&1
