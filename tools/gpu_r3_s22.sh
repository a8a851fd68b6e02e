# checkpoint: full GPU suite, smoke, host-side cProfile of the C2 step
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r3s22}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -rf > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 300 python -u tools/host_profile2.py > $OUT/host_profile.log 2>&1 || exit 1
head -70 $OUT/host_profile.log
