"""Is the 8192 x 4096 x 512 input-projection GEMM (decoder lstm2 layer 0) bound by its output
stores?  Times it with an fp32 C, a bf16-only C and an fp32 C + bf16 twin (HIP events).
    python tools/store_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import autoformer_amd as A  # noqa: E402
from autoformer_amd import kernels as K  # noqa: E402


def t(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


A.set_compute("bf16")
for M, N, Kd in ((8192, 4096, 512), (8192, 1024, 4096), (8192, 4096, 64)):
    a = torch.randn(M, Kd, device="cuda").bfloat16()
    b = torch.randn(N, Kd, device="cuda").bfloat16()
    c32 = torch.empty(M, N, device="cuda")
    c16 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    bias = torch.randn(N, device="cuda")
    us32 = t(lambda: K.gemm(M, N, Kd, K.operand(a, Kd), K.operand(b, Kd), c32, bias=bias))
    us16 = t(lambda: K.gemm(M, N, Kd, K.operand(a, Kd), K.operand(b, Kd), c16, bias=bias))
    usb = t(lambda: K.gemm(M, N, Kd, K.operand(a, Kd), K.operand(b, Kd), c32, bias=bias, c_bf16=c16))
    mb = M * N * 4 / 1e6
    print(f"{M}x{N}x{Kd}: fp32 C {us32:7.1f} us ({mb / us32:5.2f} TB/s of C)  bf16 C {us16:7.1f} us  "
          f"fp32 + bf16 twin {usb:7.1f} us", flush=True)
