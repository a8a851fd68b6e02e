# token-mixing products on the NT kernel: tests, census lines, C4 / MetaPool bench
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r3s35}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
timeout -k 10 800 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_metaformer.py tests/test_variants.py tests/test_gpu_model.py tests/test_gpu_capture.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 400 python -u tools/gemm_census.py --model MetaConv --reps 5 > $OUT/census.txt 2>&1 || exit 1
grep -E "344x7424x1856|1856x7424|7424x1856" $OUT/census.txt
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --model MetaConv --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> $OUT/bench.log || exit 1
  timeout -k 10 300 python -u bench.py --model MetaPool --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> $OUT/bench.log || exit 1
done
cat $OUT/bench.log
