set -o pipefail
cd $GRAFT_REPO_ROOT
echo "== MetaConv"; bash tools/ab_head.sh "--model MetaConv --steps 10 --warmup 3" "AVC_GELU_FUSE=0" 2 || exit 1
echo "== C2"; bash tools/ab_head.sh "--steps 30 --warmup 5" "" 2 || exit 1
