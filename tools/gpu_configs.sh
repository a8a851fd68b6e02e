# the other BASELINE configs on one box (C4 MetaConv, MetaPool, C5 AutoVC + Discriminator; C2 again for the box)
# -> gpurun_out/$1/configs.jsonl
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-configs}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for args in "" "--model MetaConv" "--model MetaPool" "--disc"; do
  timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-kernel-timing $args \
      >> $OUT/configs.jsonl 2> $OUT/configs.err || exit 1
done
cat $OUT/configs.jsonl | python3 -c "import sys, json; [print(d['config'].get('model', d['config'].get('workload')), d['ms_per_step'], d['value']) for d in map(json.loads, sys.stdin)]"
