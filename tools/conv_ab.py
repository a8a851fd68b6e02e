"""Conv GEMM configurations (AVC_CONV_CFG) on the AutoVC conv shapes, event-timed in isolation:
  AVC_CONV_CFG=13,32,64 python tools/conv_ab.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import autoformer_amd as A  # noqa: E402
from autoformer_amd import kernels as K  # noqa: E402

A.set_compute("bf16")
dev = "cuda:0"


def ev(fn, n=50):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


cfg = os.environ.get("AVC_CONV_CFG", "default")
for B, T, Ci, Co, bn in [(64, 128, 512, 512, True), (64, 128, 512, 512, False), (64, 128, 512, 80, False),
                         (64, 176, 512, 512, True), (64, 128, 96, 512, True)]:
    M = B * T
    x = torch.randn(M, Ci, device=dev).bfloat16()
    w = (torch.randn(Co, 5 * Ci, device=dev) * 0.05).bfloat16()
    y = torch.empty(M, Co, device=dev)
    if bn:
        part = K.bn_partial_buffer(M, Co, dev)
        g, b = torch.ones(Co, device=dev), torch.zeros(Co, device=dev)
        rm, rv = torch.zeros(Co, device=dev), torch.ones(Co, device=dev)
        fn = lambda: K.gemm(M, Co, 5 * Ci, K.operand(x, Ci, window=(5, 2, T, T, Ci)), K.operand(w, 5 * Ci), y,  # noqa
                            bn_partial=part, bn_fin=(g, b, rm, rv, None, 0.1, 1e-5, 1))
    else:
        fn = lambda: K.gemm(M, Co, 5 * Ci, K.operand(x, Ci, window=(5, 2, T, T, Ci)), K.operand(w, 5 * Ci), y)  # noqa
    us = ev(fn)
    print(f"cfg {cfg}: conv B{B} T{T} {Ci}->{Co} bn={bn}: {us:6.1f} us = {2 * M * Co * 5 * Ci / us / 1e6:5.0f} TF",
          flush=True)
