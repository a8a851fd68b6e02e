# round 4: host enqueue vs GPU step (C2), per-phase host split and a cProfile of the host side -> gpurun_out/$1
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
timeout -k 10 200 python -u tools/host_time.py --steps 30 > $OUT/host_time.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/host_split.py > $OUT/host_split.txt 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/c2.json 2>/dev/null || exit 1
tail -3 $OUT/host_time.txt
head -5 $OUT/host_split.txt
grep -o '"ms_per_step": [0-9.]*' $OUT/*.json
