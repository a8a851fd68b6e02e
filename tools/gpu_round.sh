# One GPU call: parity tests, LSTM step timeline, bench line, kernel-trace stats, HBM PMC
# passes -> gpurun_out/$1.   gpurun --timeout 1100 -- bash tools/gpu_round.sh <tag> [skip-tests] [no-pmc]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-run}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  (cd $R && timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > $OUT/pytest_gpu.log 2>&1) || { tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
timeout -k 10 120 python $R/tools/lstm_trace.py > $OUT/lstm_trace.log 2>&1 &&
cat $OUT/lstm_trace.log &&
timeout -k 10 300 python $R/bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err &&
cat $OUT/bench.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit 1
if [ "$3" != "no-pmc" ]; then
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
      python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1 &&
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
      python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_write.log 2>&1 &&
  python3 $R/tools/pmc_traffic.py $OUT/pmc_fetch/run_counter_collection.csv \
      $OUT/pmc_write/run_counter_collection.csv $OUT/pmc_traffic.json || exit 1
fi
exit 0
