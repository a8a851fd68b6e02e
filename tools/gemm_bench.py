"""Microbenchmark of avc_gemm shapes on the AutoVC path (HIP events, current stream)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import autoformer_amd as A
from autoformer_amd import kernels as K

A.set_compute("bf16")
dev = "cuda:0"


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def case(name, M, N, K_, adt, bdt, aks=False, bks=False, win=None, split=1):
    a = torch.randn((K_, M) if aks else (M, K_), device=dev).to(adt)
    b = torch.randn((K_, N) if bks else (N, K_), device=dev).to(bdt)
    c = torch.empty(M, N, device=dev)
    if win is not None:
        B, T, Cin, Kw, pad = win
        a = torch.randn(B * T, Cin, device=dev).to(adt)
        opa = K.operand(a, Cin, window=(Kw, pad, T, T, Cin))
    else:
        opa = K.operand(a, M if aks else K_, kstrided=aks)
    opb = K.operand(b, N if bks else K_, kstrided=bks)
    us = timeit(lambda: K.gemm(M, N, K_, opa, opb, c, split_k=split))
    print(f"{name:40s} M={M:5d} N={N:5d} K={K_:5d}  {us:8.1f} us  {2*M*N*K_/us/1e6:7.1f} TFLOP/s", flush=True)


bf, f32 = torch.bfloat16, torch.float32
case("plain bf16/bf16 NT", 8192, 512, 2560, bf, bf)
case("plain f32/bf16 NT", 8192, 512, 2560, f32, bf)
case("plain f32/f32 NT", 8192, 512, 2560, f32, f32)
case("conv win f32 A", 8192, 512, 2560, f32, bf, win=(64, 128, 512, 5, 2))
case("conv win bf16 A", 8192, 512, 2560, bf, bf, win=(64, 128, 512, 5, 2))
case("xproj lstm2 f32 A", 8192, 4096, 1024, f32, bf)
case("xproj lstm2 bf16 A", 8192, 4096, 1024, bf, bf)
case("wgrad TT f32", 512, 2560, 8192, f32, f32, aks=True, bks=True, split=3)
case("wgrad TT bf16", 512, 2560, 8192, bf, bf, aks=True, bks=True, split=3)
case("wgrad TT f32 nosplit", 512, 2560, 8192, f32, f32, aks=True, bks=True)
case("dx NT(kstrided B) f32", 8192, 1024, 4096, f32, bf, bks=True)
case("big square bf16", 4096, 4096, 4096, bf, bf)
case("xproj lstm1 bf16 A", 8192, 2048, 344, bf, bf)
case("dgrad conv bf16", 8192, 512, 2560, bf, bf, win=(64, 128, 512, 5, 2))
case("postnet last conv bf16", 8192, 80, 2560, bf, bf, win=(64, 128, 512, 5, 2))
case("postnet first conv bf16", 8192, 512, 400, bf, bf, win=(64, 128, 80, 5, 2))


def torch_case(name, M, N, K_):
    a = torch.randn(M, K_, device=dev).to(bf)
    b = torch.randn(N, K_, device=dev).to(bf)
    us = timeit(lambda: torch.matmul(a, b.t()))
    print(f"{'hipBLASLt ' + name:40s} M={M:5d} N={N:5d} K={K_:5d}  {us:8.1f} us  {2*M*N*K_/us/1e6:7.1f} TFLOP/s", flush=True)


torch_case("conv-shaped", 8192, 512, 2560)
torch_case("xproj lstm2", 8192, 4096, 1024)
torch_case("wgrad-shaped", 512, 2560, 8192)
torch_case("big square", 4096, 4096, 4096)
torch_case("lstm2 W_ih wgrad", 4096, 1024, 8192)
