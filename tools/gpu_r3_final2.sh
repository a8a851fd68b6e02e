# round-3 closing pass: full GPU suite + smoke, then the measurement pass (tools/gpu_r3_final.sh)
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r3final2}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -rf > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
bash $R/tools/gpu_r3_final.sh $T || exit 1
