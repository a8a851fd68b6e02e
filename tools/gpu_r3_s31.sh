# fused BN backward, all partial rows in flight in the finalize: tests, kernel time, A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r3s31}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_capture.py -k "bn or capture" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
cd /tmp && export TMPDIR=/tmp
for f in 1 0; do
AVC_BN_BWD_FUSE=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof$f -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing > $OUT/prof$f.log 2>&1 || exit 1
CSV=$(find $OUT/prof$f -name "run_kernel_trace.csv" | head -1)
python3 $R/tools/step_breakdown.py $CSV 30 > $OUT/breakdown$f.txt
echo "== fuse $f"; grep -i "bn_\|span\|busy" $OUT/breakdown$f.txt | head -12
done
cd $R
for r in 1 2 3 4; do
  for f in 1 0; do
    echo -n "fuse $f rep $r: " >> $OUT/ab.log
    AVC_BN_BWD_FUSE=$f timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> $OUT/ab.log || exit 1
  done
done
cat $OUT/ab.log
