set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/r3t.log
for cfg in "1 1" "16 0"; do
set -- $cfg
echo "segments $1 serial $2" >> $O
AVC_GRAPH_SEGMENTS=$1 AVC_GRAPH_SERIAL=$2 timeout -k 10 200 python -u tools/graph_debug4.py bf16 > gpurun_out/r3t_tmp.log 2>&1 || exit 1
grep "split\|single" gpurun_out/r3t_tmp.log >> $O
done
