set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r3s18}
bash $R/tools/gpu_r3_s15.sh $T || exit 1
bash $R/tools/gpu_r3_s17.sh $T || exit 1
bash $R/tools/gpu_r3_s14.sh $T || exit 1
