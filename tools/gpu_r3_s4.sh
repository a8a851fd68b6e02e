set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r3s4}
mkdir -p $OUT
for v in "AVC_GRAPH_SERIAL=1 AVC_GRAPH_SEGMENTS=1" "AVC_GRAPH_SERIAL=1 AVC_GRAPH_SEGMENTS=2" "AVC_GRAPH_SERIAL=1 AVC_GRAPH_RUNS=1" "AVC_GRAPH_RUNS=1"; do
  echo "== $v" >> $OUT/graph_check.log
  env $v timeout -k 10 150 python -u tools/graph_check.py 3 >> $OUT/graph_check.log 2>&1 || exit 1
done
echo "== bench RUNS=1" >> $OUT/graph_check.log
AVC_GRAPH_RUNS=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --graph --no-cpu-baseline --no-kernel-timing 2>/dev/null | cut -c1-200 >> $OUT/graph_check.log
