# BN kernel tests, then C2 bench for the finalize variants (fused fwd / last-block bwd on/off)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -k "bn or bf16 or model" > gpurun_out/t_k.log 2>&1 || exit 1
B="timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline"
$B > gpurun_out/bench_h11.log 2>&1 || exit 1
AVC_GEMM_BNFIN=0 $B > gpurun_out/bench_h01.log 2>&1 || exit 1
AVC_LAST_BLOCK=0 $B > gpurun_out/bench_h10.log 2>&1 || exit 1
AVC_GEMM_BNFIN=0 AVC_LAST_BLOCK=0 $B > gpurun_out/bench_h00.log 2>&1 || exit 1
$B > gpurun_out/bench_h11b.log 2>&1
