# round 4: MetaFormer tests + capture, C4 / MetaPool / C2 benches, C4 breakdown -> gpurun_out/$1
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_metaformer.py tests/test_gpu_capture.py tests/test_gpu_kernels.py -x -q --timeout 600 --timeout-method thread \
    > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --model MetaConv --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c4.$rep.json 2>/dev/null || exit 1
done
timeout -k 10 200 python -u bench.py --model MetaPool --steps 10 --warmup 3 --no-cpu-baseline > $OUT/mp.json 2>/dev/null || exit 1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/c2.json 2>/dev/null || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o run -- \
    python3 $R/bench.py --model MetaConv --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > $OUT/prof_c4.log 2>&1 || exit 1
python3 $R/tools/step_breakdown.py $OUT/prof_c4/run_kernel_trace.csv 60 > $OUT/prof_c4_breakdown.txt 2>&1
rm -rf $OUT/prof_c4
grep -o '"ms_per_step": [0-9.]*' $OUT/*.json
