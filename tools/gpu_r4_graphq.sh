# round 4: hipGraph replay with parallel graph queues (DEBUG_HIP_FORCE_GRAPH_QUEUES) vs eager -> gpurun_out/$1
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/eager.json 2>/dev/null || exit 1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --graph > $OUT/graph_q0.json 2>$OUT/graph_q0.err || exit 1
for q in 2 4 8; do
  DEBUG_HIP_FORCE_GRAPH_QUEUES=$q timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --graph \
      > $OUT/graph_q$q.json 2>$OUT/graph_q$q.err || exit 1
done
grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.e+]*' $OUT/*.json
