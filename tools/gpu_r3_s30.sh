# BN backward reduce + finalize fused with 16-B write-through partials: tests, interleaved A/B, profile
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r3s30}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_capture.py tests/test_gpu_model.py tests/test_gpu_graph.py -k "bn or capture or model or golden or graph" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for r in 1 2 3 4; do
  for f in 1 0; do
    echo -n "fuse $f rep $r: " >> $OUT/ab.log
    AVC_BN_BWD_FUSE=$f timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> $OUT/ab.log || exit 1
  done
done
cat $OUT/ab.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing > $OUT/prof.log 2>&1 || exit 1
CSV=$(find $OUT/prof -name "run_kernel_trace.csv" | head -1)
python3 $R/tools/step_breakdown.py $CSV 30 > $OUT/breakdown.txt
grep -i "bn_" $OUT/breakdown.txt
