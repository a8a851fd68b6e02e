# kernel-trace profiles of the C2 bench, fused BN (p_bn1) and separate finalize (p_bn0)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_prof.sh p_bn1 || exit 1
AVC_BN_FUSED=0 bash tools/gpu_prof.sh p_bn0
