# Round-6 check: full GPU suite, then an interleaved A/B of environment settings on the C2 bench
#   gpurun -- bash tools/gpu_r6_check.sh <tag> <rounds> "<envA>" "<envB>" ...
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
TAG=$1
ROUNDS=$2
shift 2
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
bash tools/gpu_ab.sh $TAG $ROUNDS "$@"
