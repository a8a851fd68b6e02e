set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_r3_s15.sh ${1:-r3s16} || exit 1
bash $R/tools/gpu_r3_s14.sh ${1:-r3s16} || exit 1
