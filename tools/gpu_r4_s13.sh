# round 4: ring / capture / metaformer tests, C4 census with epilogue ablations, C4 / MetaPool / C2 benches -> gpurun_out/$1
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
    > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u tools/gemm_census.py --model MetaConv --reps 5 --strip 'col_sum;act_grad_of' > $OUT/census_c4_strip.txt 2>&1 || { tail -20 $OUT/census_c4_strip.txt; exit 1; }
grep gelu $OUT/census_c4_strip.txt | head -16
timeout -k 10 300 python -u tools/gemm_census.py --model AutoVC --reps 10 > $OUT/census_c2.txt 2>&1 || { tail -20 $OUT/census_c2.txt; exit 1; }
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --model MetaConv --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c4.$rep.json 2>/dev/null || exit 1
done
timeout -k 10 200 python -u bench.py --model MetaPool --steps 10 --warmup 3 --no-cpu-baseline > $OUT/mp.json 2>/dev/null || exit 1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/c2.json 2>/dev/null || exit 1
grep -o '"ms_per_step": [0-9.]*' $OUT/*.json
