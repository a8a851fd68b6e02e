#!/bin/bash
# rocprofv3 kernel statistics of the MetaConv step (BASELINE config C4: B=64, T=176, bf16).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_MetaConv -o run -- \
  python3 $R/bench.py --model MetaConv --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_MetaConv.log 2>&1
