#!/bin/bash
# GPU round for the model variants: parity tests, then one bench line per variant.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_variants.py -v -m gpu --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_variants.log 2>&1 || exit 1
for m in AutoVC2 AutoVC_Adjust MetaConv2 MetaPool2 MetaConv_Adjust MetaPool_Adjust; do
  timeout -k 10 300 python -u bench.py --model $m --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/bench_$m.log 2>&1 || exit 1
done
