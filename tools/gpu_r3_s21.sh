# Discriminator conv3 padded gradients + dense backward: tests, C5 census/bench/profile, BiLSTM phases
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r3s21}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "disc_dense or pack_slice or fold" > $OUT/k_tests.log 2>&1 || { tail -30 $OUT/k_tests.log; exit 1; }
tail -2 $OUT/k_tests.log
timeout -k 10 300 python -u -m pytest -q -m gpu --timeout 250 --timeout-method thread -rf tests/test_gpu_disc.py > $OUT/disc_tests.log 2>&1 || { tail -30 $OUT/disc_tests.log; exit 1; }
tail -2 $OUT/disc_tests.log
AVC_GEMM_TRACE=1 timeout -k 10 200 python -u bench.py --disc --steps 1 --warmup 1 --no-cpu-baseline > $OUT/trace_disc.json 2> $OUT/trace_disc.err || exit 1
sort $OUT/trace_disc.err | uniq -c | grep "avc_gemm generic" || true
for r in 1 2; do
timeout -k 10 300 python -u bench.py --disc --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> $OUT/bench_disc.log || exit 1
done
cat $OUT/bench_disc.log
timeout -k 10 120 python -u tools/lstm_trace.py > $OUT/trace.log 2>&1 || exit 1
grep BiLSTM $OUT/trace.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_disc -o run -- python3 $R/bench.py --disc --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing > $OUT/prof_disc.log 2>&1 || exit 1
CSV=$(find $OUT/prof_disc -name "run_kernel_trace.csv" | head -1)
python3 $R/tools/step_breakdown.py $CSV 60 > $OUT/breakdown_disc.txt
head -30 $OUT/breakdown_disc.txt
