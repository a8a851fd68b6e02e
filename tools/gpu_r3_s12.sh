set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r3s12}
mkdir -p $OUT
cd $R
timeout -k 10 200 python -u tools/host_profile2.py > $OUT/host2.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -q --timeout 250 --timeout-method thread -rf tests/test_gpu_model.py tests/test_gpu_graph.py > $OUT/model.log 2>&1; echo "rc $?" >> $OUT/model.log
tail -3 $OUT/model.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_disc -o run -- \
      python3 $R/bench.py --disc --steps 8 --warmup 3 --no-cpu-baseline > $OUT/prof_disc.log 2>&1 || exit 1
CSV=$(find $OUT/prof_disc -name "run_kernel_trace.csv" | head -1)
python3 $R/tools/step_breakdown.py $CSV 40 > $OUT/breakdown_disc.txt 2>&1
