# round 4: ring + full GPU suite, C2 / C4 / C5 benches, C2 / C4 kernel-trace breakdowns -> gpurun_out/$1
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_ring.py -x -q --timeout 120 --timeout-method thread \
    > $OUT/ring_tests.log 2>&1 || { tail -30 $OUT/ring_tests.log; exit 1; }
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rA \
      > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/c2.$rep.json 2>/dev/null || exit 1
  timeout -k 10 200 python -u bench.py --model MetaConv --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c4.$rep.json 2>/dev/null || exit 1
done
timeout -k 10 200 python -u bench.py --disc --steps 20 --warmup 3 --no-cpu-baseline > $OUT/c5.json 2>/dev/null || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing > $OUT/prof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o run -- \
    python3 $R/bench.py --model MetaConv --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > $OUT/prof_c4.log 2>&1 || exit 1
for d in prof prof_c4; do
  python3 $R/tools/step_breakdown.py $OUT/$d/run_kernel_trace.csv 40 > $OUT/${d}_breakdown.txt 2>&1
  cp $OUT/$d/run_kernel_stats.csv $OUT/${d}_kernel_stats.csv 2>/dev/null
  rm -rf $OUT/$d
done
grep -o '"ms_per_step": [0-9.]*' $OUT/*.json
