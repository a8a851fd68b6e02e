# fold margins / parity / rocprof A/B, graph ordering experiment, 256-row conv tiles A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3s10}
bash $R/tools/gpu_r3_s8.sh $TAG || exit 1
cd $R
bash $R/tools/gpu_r3_s9.sh $TAG || exit 1
