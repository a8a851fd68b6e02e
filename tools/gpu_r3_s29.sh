# zero_grad on the side stream vs on the main stream: interleaved A/B (AVC_ZERO_SIDE), host time of each
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r3s29}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
for r in 1 2 3 4; do
  for z in 1 0; do
    echo -n "zero_side $z rep $r: " >> $OUT/ab.log
    AVC_ZERO_SIDE=$z timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> $OUT/ab.log || exit 1
  done
done
for z in 1 0; do AVC_ZERO_SIDE=$z timeout -k 10 200 python -u tools/host_time.py 2>/dev/null | grep host >> $OUT/ab.log || exit 1; done
cat $OUT/ab.log
