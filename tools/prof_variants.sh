#!/bin/bash
# rocprofv3 kernel statistics of the AutoVC2 and AutoVC_Adjust steps (B=64, T=128, bf16).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for m in AutoVC2 AutoVC_Adjust; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$m -o run -- \
    python3 $R/bench.py --model $m --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_$m.log 2>&1 || exit 1
done
