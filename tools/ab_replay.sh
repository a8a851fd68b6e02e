# interleaved bench.py --replay A/B over env configs: bash tools/ab_replay.sh <outdir> "<cfg1>" "<cfg2>" ...
OUT=gpurun_out/$1; shift
mkdir -p $OUT
for i in 1 2; do
 for cfg in "$@"; do
  env $cfg timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --replay > /tmp/o.json 2>/dev/null || exit 1
  echo "$cfg $(grep -o 'ms_per_step": [0-9.]*' /tmp/o.json)" >> $OUT/ab.txt
 done
done
cat $OUT/ab.txt
