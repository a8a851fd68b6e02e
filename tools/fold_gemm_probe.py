"""Probe: the decoder lstm1 fold's small GEMMs (AutoVC C2 shapes: B = 64, nc = 8, cd = 88, de =
256, G = 2048) alone on the GPU, fp32 operand A (the fast generic kernel) against a bf16 A (the
NT / ring kernels), plus expand_codes and segsum -- the serial chain between the BiLSTM and the
lstm1 recurrence (forward) and after it (backward).

  python tools/fold_gemm_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from autoformer_amd import kernels as K
from autoformer_amd.kernels import operand


def timed(fn, reps=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    K.set_compute("bf16")
    dev = torch.device("cuda:0")
    B, nc, cd, de, H, T = 64, 8, 88, 256, 512, 128
    G, In = 4 * H, cd + de
    g = torch.Generator(device=dev).manual_seed(0)
    codes = torch.randn(B * nc, cd, device=dev, generator=g)
    codes16 = codes.to(torch.bfloat16)
    emb = torch.randn(B, de, device=dev, generator=g)
    emb16 = emb.to(torch.bfloat16)
    wih = (torch.randn(G, In, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    wih_t = wih.t().contiguous()
    bsum = torch.randn(G, device=dev, generator=g)
    pc = torch.empty(B * nc, G, device=dev)
    pe = torch.empty(B, G, device=dev)
    res = {}
    res["pc fp32 A"] = timed(lambda: K.gemm(B * nc, G, cd, operand(codes, cd), operand(wih, In), pc))
    res["pc bf16 A"] = timed(lambda: K.gemm(B * nc, G, cd, operand(codes16, cd), operand(wih, In), pc))
    res["pe fp32 A"] = timed(lambda: K.gemm(B, G, de, operand(emb, de), operand(wih[:, cd:], In), pe, bias=bsum))
    res["pe bf16 A"] = timed(lambda: K.gemm(B, G, de, operand(emb16, de), operand(wih[:, cd:], In), pe, bias=bsum))
    res["expand_codes"] = timed(lambda: K.expand_codes(pc, pe, B, T, nc))
    dg = torch.randn(B * T, G, device=dev, generator=g)
    res["segsum code"] = timed(lambda: K.segsum(dg, B * nc, T // nc, G, ld=G))
    s_code = K.segsum(dg, B * nc, T // nc, G, ld=G)
    s16 = s_code.to(torch.bfloat16)
    dcodes = torch.empty(B * nc, cd, device=dev)
    sk = K.auto_split_k(B * nc, cd, G)
    res[f"dcodes fp32 A split {sk}"] = timed(lambda: K.gemm(B * nc, cd, G, operand(s_code, G), operand(wih_t, G),
                                                            dcodes, split_k=sk))
    res[f"dcodes bf16 A split {sk}"] = timed(lambda: K.gemm(B * nc, cd, G, operand(s16, G), operand(wih_t, G),
                                                            dcodes, split_k=sk))
    res["dcodes fp32 A split 1"] = timed(lambda: K.gemm(B * nc, cd, G, operand(s_code, G), operand(wih_t, G), dcodes))
    for k, v in res.items():
        print(f"{k:28s} {v:8.2f} us")


if __name__ == "__main__":
    main()
