# three back-to-back default bench runs on one box (box-to-box spread check)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/bench3; mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 300 python $R/bench.py > $OUT/b$i.json 2> $OUT/b$i.err || { tail $OUT/b$i.err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $OUT/b$i.json
done
