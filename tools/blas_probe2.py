"""NN products of the C2 / C4 steps: the ring kernel (kernels.gemm, default policy) against the
vendor BLAS torch.matmul dispatches to (hipBLASLt on ROCm) on the same bf16 operands -- what a
tuned library reaches on each shape, i.e. the headroom of the hand-written kernel.
python tools/blas_probe2.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import autoformer_amd as A  # noqa: E402
from autoformer_amd import kernels as K  # noqa: E402

A.set_compute("bf16")
dev = "cuda:0"


def ev(fn, n=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


SHAPES = [(22016, 7424, 1856, "C4 token FF1"), (22016, 1856, 7424, "C4 token FF2 / dY1T"),
          (118336, 1376, 344, "C4 channel FF1"), (118336, 344, 1376, "C4 channel FF2 / dY2"),
          (8192, 4096, 512, "C2 lstm2 x-projection"), (8192, 1024, 4096, "C2 lstm dX"),
          (8192, 512, 4096, "C2 lstm1 dX"), (8192, 2048, 344, "C2 lstm1 x-projection")]


def main():
    for M, N, Kd, what in SHAPES:
        a = torch.randn(M, Kd, device=dev).bfloat16()
        b = torch.randn(N, Kd, device=dev).bfloat16()
        c = torch.empty(M, N, device=dev)
        c16 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        t_ring = ev(lambda: K.gemm(M, N, Kd, K.operand(a, Kd), K.operand(b, Kd), c16))
        t_ring32 = ev(lambda: K.gemm(M, N, Kd, K.operand(a, Kd), K.operand(b, Kd), c))
        bt = b.t()
        t_blas = ev(lambda: torch.matmul(a, bt, out=c16))
        fl = 2.0 * M * N * Kd
        print(f"{what:24s} {M}x{N}x{Kd}: ring bf16-out {t_ring:7.1f} us ({fl / t_ring / 1e6:6.1f} TF)  fp32-out "
              f"{t_ring32:7.1f} us | torch.matmul (hipBLASLt) bf16-out {t_blas:7.1f} us ({fl / t_blas / 1e6:6.1f} TF)",
              flush=True)


if __name__ == "__main__":
    main()
