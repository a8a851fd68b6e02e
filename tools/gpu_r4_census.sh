# round 4: per-call GEMM census of the C4 / C2 steps, ring policy vs off vs forced tiles -> gpurun_out/$1
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u tools/gemm_census.py --model MetaConv --reps 5 --ring-ab \
    --force "256,256,2;256,128,3;128,128,4;256,256,14;256,128,15;128,128,16" > $OUT/census_c4.txt 2>&1 || { tail -20 $OUT/census_c4.txt; exit 1; }
timeout -k 10 300 python -u tools/gemm_census.py --model AutoVC --reps 10 --ring-ab \
    --force "256,256,2;256,128,3;128,128,4;256,256,14;256,128,15;128,128,16" > $OUT/census_c2.txt 2>&1 || { tail -20 $OUT/census_c2.txt; exit 1; }
tail -2 $OUT/census_c4.txt $OUT/census_c2.txt
