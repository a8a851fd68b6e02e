# kernel-trace profile of the C2 bench -> gpurun_out/$1 (CSV), plus step breakdown / gaps;
# further arguments go to bench.py (e.g. --eager)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing "$@" > $OUT/prof.log 2>&1 || exit 1
CSV=$(find $OUT/prof -name "run_kernel_trace.csv" | head -1)
python3 $R/tools/step_breakdown.py $CSV 25 > $OUT/breakdown.txt
Q=$(python3 - "$CSV" <<'PY'
import csv, sys, collections
c = collections.Counter(int(r["Queue_Id"]) for r in csv.DictReader(open(sys.argv[1])) if "lstm_persist" in r["Kernel_Name"])
print(c.most_common(1)[0][0])
PY
)
python3 $R/tools/gaps.py $CSV $Q > $OUT/gaps.txt
STATS=$(find $OUT/prof -name "run_kernel_stats.csv" | head -1)
cp $STATS $OUT/kernel_stats.csv
