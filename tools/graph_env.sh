# hipGraph replay of the C2 step under the runtime's graph-queue settings
cd $GRAFT_REPO_ROOT
for q in 1 2 4; do
  echo "DEBUG_HIP_FORCE_GRAPH_QUEUES=$q"
  DEBUG_HIP_FORCE_GRAPH_QUEUES=$q timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --graph --no-cpu-baseline --no-kernel-timing 2>/dev/null | cut -c1-200
done
echo "PACKET_CAPTURE"
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --graph --no-cpu-baseline --no-kernel-timing 2>/dev/null | cut -c1-200
