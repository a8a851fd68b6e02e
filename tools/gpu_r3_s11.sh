set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r3s11}
mkdir -p $OUT
cd $R
for f in 1 0; do echo "== FOLD=$f" >> $OUT/margin.log; AVC_CONV0_FOLD=$f timeout -k 10 120 python -u tools/bf16_margin.py >> $OUT/margin.log 2>&1 || exit 1; done
bash $R/tools/gpu_r3_s9.sh ${1:-r3s11} || exit 1
cd /tmp && export TMPDIR=/tmp
for f in 1 0; do
  AVC_CONV0_FOLD=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_fold$f -o run -- \
      python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_fold$f.log 2>&1 || exit 1
  CSV=$(find $OUT/prof_fold$f -name "run_kernel_trace.csv" | head -1)
  python3 $R/tools/step_breakdown.py $CSV 30 > $OUT/breakdown_fold$f.txt 2>&1
done
