set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r3s13}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread -rf \
  tests/test_gpu_model.py tests/test_gpu_graph.py tests/test_gpu_dist.py tests/test_gpu_disc.py tests/test_variants.py \
  tests/test_gpu_fullsize.py tests/test_gpu_capture.py tests/test_gpu_fold.py > $OUT/tests.log 2>&1; rc=$?
tail -4 $OUT/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 200 python -u tools/host_time.py --steps 20 > $OUT/host_time.log 2>&1 || exit 1
cat $OUT/host_time.log | grep -v amdgpu
for r in 1 2 3; do
timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline 2>/dev/null | cut -c1-200 >> $OUT/bench.log || exit 1
done
grep -o '"ms_per_step": [0-9.]*' $OUT/bench.log
