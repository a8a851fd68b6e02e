# Same-box A/B of environment settings on the bench step: gpu_envab.sh <tag> "ENV=a ENV2=b" "ENV=c" ...
# each setting runs twice, interleaved (a b a b) -> gpurun_out/<tag>/ab.txt
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-envab}
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for rep in $(seq 1 ${AB_REPS:-2}); do
  i=0
  for spec in "$@"; do
    i=$((i+1))
    env $spec timeout -k 10 200 python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-kernel-timing \
        > $OUT/b_${i}_$rep.json 2> $OUT/b_${i}_$rep.err || { tail $OUT/b_${i}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/b_${i}_$rep.json')); print('[$spec]', d['ms_per_step'], d['value'])" | tee -a $OUT/ab.txt
  done
done
