# kernel-trace profiles of the C2 bench: lstm1 fold (p_f1) and concat path (p_f0)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_prof.sh p_f1 || exit 1
AVC_FOLD=0 bash tools/gpu_prof.sh p_f0
