# BN micro-bench (fused / separate finalize), BN + model tests, C2 bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/bn_bench.py > gpurun_out/bn_bench.log 2>&1 || exit 1
AVC_BN_FUSED=0 timeout -k 10 120 python -u tools/bn_bench.py >> gpurun_out/bn_bench.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_disc.py -m gpu -k "bn or model or disc" > gpurun_out/t_bn.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_bn1.log 2>&1 || exit 1
AVC_BN_FUSED=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_bn0.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_bn1b.log 2>&1
