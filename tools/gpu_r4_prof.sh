# round 4: kernel-trace breakdowns of the C4 and C5 steps -> gpurun_out/$1
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o run -- \
    python3 $R/bench.py --model MetaConv --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > $OUT/prof_c4.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o run -- \
    python3 $R/bench.py --disc --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > $OUT/prof_c5.log 2>&1 || exit 1
for d in prof_c4 prof_c5; do
  python3 $R/tools/step_breakdown.py $OUT/$d/run_kernel_trace.csv 45 > $OUT/${d}_breakdown.txt 2>&1
  rm -rf $OUT/$d
done
head -50 $OUT/prof_c4_breakdown.txt
