# round-3 measurement pass: LSTM timeline, bench line (cpu_baseline + roofline), kernel-trace stats,
# HBM PMC passes (tools/gpu_round.sh), then the BASELINE configs C4 / MetaPool / C5 and the variants
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r3final}
OUT=$R/gpurun_out/$T
bash $R/tools/gpu_round.sh $T skip-tests || exit 1
cd $R
for m in MetaConv MetaPool; do
  timeout -k 10 300 python -u bench.py --model $m --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_$m.json 2>/dev/null || exit 1
done
timeout -k 10 300 python -u bench.py --disc --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_disc.json 2>/dev/null || exit 1
for m in AutoVC2 AutoVC_Adjust MetaConv2 MetaPool2 MetaConv_Adjust MetaPool_Adjust; do
  timeout -k 10 300 python -u bench.py --model $m --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_$m.json 2>/dev/null || exit 1
done
grep -o '"ms_per_step": [0-9.]*' $OUT/bench*.json
