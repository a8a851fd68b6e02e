"""Weight-gradient (TT) GEMM shapes of the C2 step: the library's TT kernels (auto split-K) against
hipBLASLt (torch.mm on the transposed view, bf16 out) on the same bf16 operands, isolated.

  python tools/tt_blas_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import autoformer_amd as A  # noqa: E402
from autoformer_amd import kernels as K  # noqa: E402

A.set_compute("bf16")
dev = "cuda:0"
bf = torch.bfloat16


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def case(name, M, N, Kf, win=None, splits=None):
    a = torch.randn(Kf, M, device=dev).to(bf)
    if win:
        Cin = win[4]
        b = torch.randn(Kf, Cin, device=dev).to(bf)
        opb = K.operand(b, Cin, kstrided=True, window=win)
        # the materialised im2col for hipBLASLt: column tap*Cin + c of frame f = x[f + tap - pad][c]
        taps, pad, T = win[0], win[1], win[2]
        xb = b.view(-1, T, Cin)
        cols = []
        for t in range(taps):
            sh = torch.zeros_like(xb)
            lo, hi = max(0, pad - t), min(T, T + pad - t)
            sh[:, lo:hi] = xb[:, lo + t - pad:hi + t - pad]
            cols.append(sh)
        bl = torch.cat(cols, dim=2).view(Kf, taps * Cin)
    else:
        b = torch.randn(Kf, N, device=dev).to(bf)
        opb = K.operand(b, N, kstrided=True)
        bl = b
    c = torch.empty(M, N, device=dev)
    fl = 2 * M * N * Kf
    for sk in splits or [K.auto_split_k(M, N, Kf)]:
        us = timeit(lambda: K.gemm(M, N, Kf, K.operand(a, M, kstrided=True), opb, c, split_k=sk))
        print(f"{name:30s} M={M:5d} N={N:5d} K={Kf:5d} ours split={sk:2d} {us:8.1f} us {fl / us / 1e6:7.1f} TF",
              flush=True)
    at = a.t()
    us = timeit(lambda: torch.mm(at, bl))
    print(f"{name:30s} M={M:5d} N={N:5d} K={Kf:5d} hipBLASLt         {us:8.1f} us {fl / us / 1e6:7.1f} TF", flush=True)


case("conv wgrad 512x(5*512)", 512, 2560, 8192, win=(5, 2, 128, 128, 512))
case("enc conv0 wgrad 512x(5*96)", 512, 480, 8192, win=(5, 2, 128, 128, 96))
case("postnet wgrad 80x(5*512)", 80, 2560, 8192, win=(5, 2, 128, 128, 512))
case("lstm2 dW_ih1 4096x1024", 4096, 1024, 8192)
case("lstm2 dW_hh shift 4096x1024", 4096, 1024, 8192, win=(1, 1, 128, 128, 1024))
case("lstm2 dW_ih0 4096x512", 4096, 512, 8192)
case("lstm1 dW_hh shift 2048x512", 2048, 512, 8192, win=(1, 1, 128, 128, 512))
case("bilstm dW_ih 352x512", 352, 512, 8192)
