# Interleaved same-box A/B of environment settings on the C2 bench -> gpurun_out/$1/ab.txt
#   gpurun -- bash tools/gpu_ab.sh <tag> <rounds> "<envA>" "<envB>" ...   (env "-" = defaults)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
ROUNDS=$2
shift 2
mkdir -p $OUT
for r in $(seq $ROUNDS); do
  for cfg in "$@"; do
    E=""
    [ "$cfg" != "-" ] && E="$cfg"
    line=$(env $E timeout -k 10 200 python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing 2> $OUT/err.log) || { echo "FAILED $cfg"; tail -5 $OUT/err.log; exit 1; }
    ms=$(echo "$line" | python3 -c "import sys,json; print(json.loads(sys.stdin.read())['ms_per_step'])")
    echo "round $r  [$cfg]  $ms ms" | tee -a $OUT/ab.txt
  done
done
