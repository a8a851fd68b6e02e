# kernel stats of the bench step with and without the 8-channel BN apply forms
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/s6; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  AVC_APPLY8=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p$v -o run -- \
      python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing > $OUT/p$v.log 2>&1 || exit 1
  grep ms_per_step $OUT/p$v.log | head -1
done
