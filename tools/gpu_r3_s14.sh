set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r3s14}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -q -m gpu --timeout 250 --timeout-method thread -rf tests/test_gpu_disc.py > $OUT/disc_tests.log 2>&1 || { tail -30 $OUT/disc_tests.log; exit 1; }
tail -2 $OUT/disc_tests.log
timeout -k 10 300 python -u bench.py --disc --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_disc.json 2>/dev/null || exit 1
timeout -k 10 300 python -u bench.py --model MetaConv --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_MetaConv.json 2>/dev/null || exit 1
grep -o '"ms_per_step": [0-9.]*' $OUT/bench_disc.json $OUT/bench_MetaConv.json
bash $R/tools/gpu_prof.sh ${1:-r3s14}/c2 || exit 1
head -5 $OUT/c2/breakdown.txt
