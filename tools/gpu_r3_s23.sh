# high-priority main stream (AVC_STREAM_PRIO) correctness + interleaved A/B, C2 and C5
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r3s23}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
AVC_STREAM_PRIO=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_disc.py tests/test_gpu_fullsize.py tests/test_gpu_fault.py > $OUT/prio_tests.log 2>&1 || { tail -30 $OUT/prio_tests.log; exit 1; }
tail -2 $OUT/prio_tests.log
for r in 1 2 3; do
  for p in 0 1; do
    echo -n "prio $p rep $r: " >> $OUT/prio_ab.log
    AVC_STREAM_PRIO=$p timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> $OUT/prio_ab.log || exit 1
  done
done
for r in 1 2; do
  for p in 0 1; do
    echo -n "C5 prio $p rep $r: " >> $OUT/prio_ab.log
    AVC_STREAM_PRIO=$p timeout -k 10 300 python -u bench.py --disc --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> $OUT/prio_ab.log || exit 1
  done
done
cat $OUT/prio_ab.log
