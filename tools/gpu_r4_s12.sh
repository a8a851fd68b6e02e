# round 4: C4 GEMM census with epilogue ablations (col_sum / GELU-backward input removed) -> gpurun_out/$1
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u tools/gemm_census.py --model MetaConv --reps 5 --strip 'col_sum;act_grad_of;col_sum,act_grad_of;c_bf16_act,c_bf16' > $OUT/census_c4_strip.txt 2>&1 || { tail -20 $OUT/census_c4_strip.txt; exit 1; }
grep gelu $OUT/census_c4_strip.txt | head -16
