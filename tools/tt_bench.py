"""Weight-gradient GEMM shapes of the step: TT LDS kernel vs the register-staged fast kernel."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import autoformer_amd as A
from autoformer_amd import kernels as K
A.set_compute("bf16")
dev = "cuda:0"
bf = torch.bfloat16


def timeit(fn, reps=20):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def case(name, M, N, Kf, win=None, splits=None):
    a = torch.randn(Kf, M, device=dev).to(bf)
    if win:
        Cin = win[4]
        b = torch.randn(Kf, Cin, device=dev).to(bf)
        opb = K.operand(b, Cin, kstrided=True, window=win)
    else:
        b = torch.randn(Kf, N, device=dev).to(bf)
        opb = K.operand(b, N, kstrided=True)
    c = torch.empty(M, N, device=dev)
    for sk in splits or [K.auto_split_k(M, N, Kf)]:
        us = timeit(lambda: K.gemm(M, N, Kf, K.operand(a, M, kstrided=True), opb, c, split_k=sk))
        print(f"{name:34s} M={M:5d} N={N:5d} K={Kf:5d} split={sk:2d}  {us:8.1f} us  {2*M*N*Kf/us/1e6:7.1f} TFLOP/s",
              flush=True)


SWEEP = os.environ.get("TT_SWEEP") is not None


case("conv wgrad 512x(5*512)", 512, 2560, 8192, win=(5, 2, 128, 128, 512), splits=[2, 3, 4, 5, 6, 8] if SWEEP else None)
case("postnet wgrad 512x(5*80)", 512, 400, 8192, win=(5, 2, 128, 128, 80))
case("enc conv0 wgrad 512x(5*336)", 512, 1680, 8192, win=(5, 2, 128, 128, 336), splits=[3, 4, 6, 7, 8] if SWEEP else None)
case("lstm2 dW_ih 4096x1024", 4096, 1024, 8192)
case("lstm2 dW_hh shift 4096x1024", 4096, 1024, 8192, win=(1, 1, 128, 128, 1024))
case("lstm1 dW_ih 2048x344", 2048, 344, 8192, splits=[2, 4, 6, 8] if SWEEP else None)
case("linear dW 80x1024", 80, 1024, 8192)
