# round-4 measurement pass: full GPU suite + smoke, bench line (cpu_baseline + roofline), kernel-trace
# stats, HBM PMC passes, MFMA counter pass, BASELINE configs C4 / MetaPool / C5 -> gpurun_out/$1
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r4final}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 900 --timeout-method thread -rf > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
bash $R/tools/gpu_round.sh $T skip-tests || exit 1
bash $R/tools/gpu_pmc.sh $T || exit 1
cd $R
for m in MetaConv MetaPool; do
  timeout -k 10 300 python -u bench.py --model $m --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_$m.json 2>/dev/null || exit 1
done
timeout -k 10 300 python -u bench.py --disc --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_disc.json 2>/dev/null || exit 1
rm -rf $OUT/pmc_fetch $OUT/pmc_write $OUT/step $OUT/tt
grep -o '"ms_per_step": [0-9.]*' $OUT/bench*.json
