# same-box A/B of the working tree against the HEAD copy in _ab_head/ (git archive + its own build):
#   bash tools/ab_head.sh "<bench args>" "<env for new, variant 2>" [rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT
ARGS="$1"; E2="$2"; N=${3:-2}
for i in $(seq 1 $N); do
  (cd _ab_head && timeout -k 10 300 python -u bench.py $ARGS --no-cpu-baseline --no-kernel-timing > ../gpurun_out/abh_head$i.log 2>&1) || exit 1
  echo "HEAD $(grep -ho '"ms_per_step": [0-9.]*' gpurun_out/abh_head$i.log)"
  timeout -k 10 300 python -u bench.py $ARGS --no-cpu-baseline --no-kernel-timing > gpurun_out/abh_new$i.log 2>&1 || exit 1
  echo "NEW  $(grep -ho '"ms_per_step": [0-9.]*' gpurun_out/abh_new$i.log)"
  if [ -n "$E2" ]; then
    env $E2 timeout -k 10 300 python -u bench.py $ARGS --no-cpu-baseline --no-kernel-timing > gpurun_out/abh_new2$i.log 2>&1 || exit 1
    echo "NEW[$E2] $(grep -ho '"ms_per_step": [0-9.]*' gpurun_out/abh_new2$i.log)"
  fi
done
