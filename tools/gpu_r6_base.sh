# Round-6 baseline: C2 bench line + kernel trace of the replayed step with the main-queue timeline
#   gpurun -- bash tools/gpu_r6_base.sh <tag> [bench args...]
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 python3 $R/bench.py --steps 20 --warmup 5 "$@" > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing "$@" > $OUT/prof.log 2>&1 || exit 1
CSV=$(find $OUT/prof -name "run_kernel_trace.csv" | head -1)
python3 $R/tools/step_breakdown.py $CSV 40 > $OUT/breakdown.txt
python3 $R/tools/timeline.py $CSV 1 0 > $OUT/timeline.txt
cp $(find $OUT/prof -name "run_kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
cp $CSV $OUT/trace.csv; python3 $R/tools/queues.py $CSV 0 > $OUT/queues.txt; rm -rf $OUT/prof
