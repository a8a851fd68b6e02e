set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r3s3}
mkdir -p $OUT
for v in "AVC_GRAPH_SPLIT=0" "AVC_GRAPH_SPLIT=1" "AVC_GRAPH_SERIAL=1" "AVC_GRAPH_CLONE_ONLY=1"; do
  echo "== $v" >> $OUT/graph_check.log
  env $v timeout -k 10 150 python -u tools/graph_check.py 4 >> $OUT/graph_check.log 2>&1 || exit 1
done
