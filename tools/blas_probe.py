"""Weight-gradient GEMM shapes of the AutoVC C2 step: our TT kernels (kernels.gemm, both operands
frame-major) against the vendor BLAS that torch.matmul dispatches to (hipBLASLt / rocBLAS) on the
same bf16 operands -- a probe for where a library GEMM would pay.  python tools/blas_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import autoformer_amd as A  # noqa: E402
from autoformer_amd import kernels as K  # noqa: E402

A.set_compute("bf16")
dev = "cuda:0"


def ev(fn, n=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


# (M, N, K, what): C[M][N] = sum_k A[k][M] B[k][N]
SHAPES = [(4096, 1024, 8192, "lstm2 dW_ih1 / dW_hh"), (4096, 512, 8192, "lstm2 dW_ih0"),
          (2048, 512, 8192, "lstm1 dW_hh"), (512, 2560, 8192, "conv dW (im2col K)"),
          (8192, 1024, 4096, "lstm2 dx (NT)"), (8192, 512, 2560, "conv fwd (im2col)")]
for M, N, Kd, what in SHAPES:
    a = torch.randn(Kd, M, device=dev).bfloat16()
    b = torch.randn(Kd, N, device=dev).bfloat16()
    c = torch.empty(M, N, device=dev)
    ours = ev(lambda: K.gemm(M, N, Kd, K.operand(a, M, kstrided=True), K.operand(b, N, kstrided=True), c,
                             split_k=K.auto_split_k(M, N, Kd)))
    at = a.t()
    lib = ev(lambda: torch.matmul(at, b))
    an = a.t().contiguous()  # NT layout for the library too
    lib_nt = ev(lambda: torch.matmul(an, b))
    fl = 2.0 * M * N * Kd
    print(f"{what:22s} {M}x{N}x{Kd}: ours(TT) {ours:7.1f} us {fl / ours / 1e6:6.0f} TF | torch TN {lib:7.1f} us "
          f"{fl / lib / 1e6:6.0f} TF | torch NN {lib_nt:7.1f} us {fl / lib_nt / 1e6:6.0f} TF", flush=True)
