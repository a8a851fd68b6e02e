set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r3s8}
mkdir -p $OUT
cd $R
AVC_CONV0_FOLD=1 timeout -k 10 120 python -u tools/bf16_margin.py > $OUT/margin.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -rf -m gpu \
  tests/test_gpu_model.py tests/test_variants.py tests/test_gpu_capture.py tests/test_gpu_kernels.py -k "not persistent_backward" > $OUT/model.log 2>&1; echo "model rc $?" >> $OUT/model.log
tail -4 $OUT/model.log
cd /tmp && export TMPDIR=/tmp
for f in 1 0; do
  AVC_CONV0_FOLD=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_fold$f -o run -- \
      python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_fold$f.log 2>&1 || exit 1
  CSV=$(find $OUT/prof_fold$f -name "run_kernel_trace.csv" | head -1)
  python3 $R/tools/step_breakdown.py $CSV 30 > $OUT/breakdown_fold$f.txt 2>&1
done
cd $R
for v in "AVC_GRAPH_CLONE_ONLY=2" "AVC_GRAPH_CLONE_ONLY=1"; do
  echo "== $v" >> $OUT/graph_check.log
  env $v timeout -k 10 150 python -u tools/graph_check.py 3 >> $OUT/graph_check.log 2>&1 || exit 1
done
