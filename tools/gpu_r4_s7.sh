# round 4: forward-graph tests and A/B vs eager (C2 / C4 / C5), host split -> gpurun_out/$1
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_ring.py -x -q --timeout 300 --timeout-method thread \
    > $OUT/graph_tests.log 2>&1 || { tail -30 $OUT/graph_tests.log; exit 1; }
tail -1 $OUT/graph_tests.log
for rep in 1 2; do
  for m in "" "--graph-fwd"; do
    tag=$([ -z "$m" ] && echo eager || echo gfwd)
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline $m > $OUT/c2_$tag.$rep.json 2>$OUT/c2_$tag.err || exit 1
    timeout -k 10 200 python -u bench.py --model MetaConv --steps 10 --warmup 3 --no-cpu-baseline $m > $OUT/c4_$tag.$rep.json 2>/dev/null || exit 1
    timeout -k 10 200 python -u bench.py --disc --steps 20 --warmup 3 --no-cpu-baseline $m > $OUT/c5_$tag.$rep.json 2>/dev/null || exit 1
  done
done
timeout -k 10 200 python -u tools/host_split.py --steps 20 > $OUT/host_split.txt 2>&1 || { tail -20 $OUT/host_split.txt; exit 1; }
head -4 $OUT/host_split.txt
grep -o '"ms_per_step": [0-9.]*' $OUT/*.json
bash $R/tools/gpu_r4_census.sh $1 || exit 1
