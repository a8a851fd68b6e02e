# round 4: same-box A/B of two builds (AVC_LIB_PATH=autoformer_amd/libautovc_hip_base.so vs the tree's),
# C2 / C4 benches interleaved + C2 / C4 GEMM census under each -> gpurun_out/$1
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
BASE=$R/autoformer_amd/libautovc_hip_base.so
for rep in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then export AVC_LIB_PATH=$BASE; else unset AVC_LIB_PATH; fi
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/c2.$v.$rep.json 2>/dev/null || exit 1
    timeout -k 10 200 python -u bench.py --model MetaConv --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c4.$v.$rep.json 2>/dev/null || exit 1
  done
done
for v in base new; do
  if [ $v = base ]; then export AVC_LIB_PATH=$BASE; else unset AVC_LIB_PATH; fi
  timeout -k 10 300 python -u tools/gemm_census.py --model AutoVC --reps 10 > $OUT/census_c2.$v.txt 2>&1 || exit 1
  timeout -k 10 300 python -u tools/gemm_census.py --model MetaConv --reps 5 > $OUT/census_c4.$v.txt 2>&1 || exit 1
done
grep -o '"ms_per_step": [0-9.]*' $OUT/*.json
