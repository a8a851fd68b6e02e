#!/bin/bash
# End-of-round GPU pass: full GPU suite, smoke, default bench, BASELINE configs C4/C5 and the
# model variants; every step under its own time limit, stopping at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 &&
timeout -k 10 300 python -u bench.py --model MetaConv --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_MetaConv.log 2>&1 &&
timeout -k 10 300 python -u bench.py --model MetaPool --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_MetaPool.log 2>&1 &&
timeout -k 10 300 python -u bench.py --disc --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_disc.log 2>&1 || exit 1
for m in AutoVC2 AutoVC_Adjust MetaConv2 MetaPool2 MetaConv_Adjust MetaPool_Adjust; do
  timeout -k 10 300 python -u bench.py --model $m --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/bench_$m.log 2>&1 || exit 1
done
