# round 4: ring tests + C4 / C2 census with the two-per-CU 128x128x2 ring tile -> gpurun_out/$1
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_ring.py -x -q --timeout 120 --timeout-method thread > $OUT/ring.log 2>&1 || { tail -30 $OUT/ring.log; exit 1; }
tail -1 $OUT/ring.log
timeout -k 10 400 python -u tools/gemm_census.py --model MetaConv --reps 5 --force "256,256,2;256,128,3;128,128,4;128,128,2" > $OUT/census_c4.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/gemm_census.py --model AutoVC --reps 10 --force "256,256,2;256,128,3;128,128,4;128,128,2" > $OUT/census_c2.txt 2>&1 || exit 1
echo done
