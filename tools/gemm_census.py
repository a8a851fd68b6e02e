"""Every avc_gemm call of one AutoVC train step (B=64, T=128, bf16), replayed in isolation with
HIP events: per-call time, TFLOP/s and the stream it ran on, largest first.  --ring-ab also times
each call with the ring kernels off (avc_gemm_set_ring(0)) next to the default policy.

  python tools/gemm_census.py [--model AutoVC|MetaConv] [--reps 10] [--ring-ab]
"""
import argparse
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

DT = {0: "f32", 1: "bf16"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="AutoVC")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--sweep", action="store_true", help="also time split-K 1..64 for the K-strided (TT) calls")
    ap.add_argument("--ring-ab", action="store_true")
    ap.add_argument("--force", default="", help="also time forced ring configs, e.g. '256,128,3;128,128,4'")
    ap.add_argument("--strip", default="", help="also time each call with these keyword arguments removed, "
                    "e.g. 'col_sum' or 'col_sum,act_grad_of' (an epilogue ablation; results not checked)")
    args = ap.parse_args()
    import importlib

    import autoformer_amd as A
    from autoformer_amd import _lib
    from autoformer_amd import kernels as K
    from autoformer_amd.detinit import det_init_, det_inputs
    from autoformer_amd.layers import side_stream
    from autoformer_amd.train import TrainStep

    A.set_compute("bf16")
    T, freq = (128, 16) if args.model == "AutoVC" else (176, 22)
    cls = getattr(importlib.import_module(f"autoformer_amd.factory.{args.model}"), args.model)
    m = cls(44, 256, 512, freq)
    det_init_(m)
    m = m.cuda().train()
    x, e = det_inputs(64, T)
    x, e = torch.from_numpy(x).cuda(), torch.from_numpy(e).cuda()
    ts = TrainStep(m)
    for _ in range(2):
        ts.step(x, e)
    torch.cuda.synchronize()

    calls = []
    real = K.gemm

    def rec(M, N, Kd, a, b, c, **kw):
        side = side_stream()
        on_side = side is not None and torch.cuda.current_stream() == side
        calls.append((M, N, Kd, a, b, c, kw, on_side))
        return real(M, N, Kd, a, b, c, **kw)

    K.gemm = rec
    try:
        ts.step(x, e)
    finally:
        K.gemm = real
    torch.cuda.synchronize()

    rows = []
    for (M, N, Kd, a, b, c, kw, on_side) in calls:
        def run():
            real(M, N, Kd, a, b, c, **kw)
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / args.reps * 1e3
        off = ""
        if args.ring_ab:
            _lib.call("avc_gemm_set_ring", 0, 0, 0, 0, 0, 2)
            run()
            e0.record()
            for _ in range(args.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            _lib.call("avc_gemm_set_ring", -1, 0, 0, 0, 0, 2)
            off = f" | ring off {e0.elapsed_time(e1) / args.reps * 1e3:.1f} us"
        for cfg in filter(None, args.force.split(";")):
            bm, bn, nst = map(int, cfg.split(","))
            _lib.call("avc_gemm_set_ring", 1, bm, bn, nst, 0, 2)
            run()
            e0.record()
            for _ in range(args.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            _lib.call("avc_gemm_set_ring", -1, 0, 0, 0, 0, 2)
            off += f" | {bm}x{bn}x{nst} {e0.elapsed_time(e1) / args.reps * 1e3:.1f}"
        for group in filter(None, args.strip.split(";")):
            drop = set(group.split(","))
            if not drop & set(k for k, v in kw.items() if v is not None):
                continue
            kw2 = {k: v for k, v in kw.items() if k not in drop}
            real(M, N, Kd, a, b, c, **kw2)
            e0.record()
            for _ in range(args.reps):
                real(M, N, Kd, a, b, c, **kw2)
            e1.record()
            torch.cuda.synchronize()
            off += f" | -{group} {e0.elapsed_time(e1) / args.reps * 1e3:.1f}"
        batch = kw.get("batch", 1)
        fl = 2.0 * M * N * Kd * batch
        lay = ("T" if a.kstrided else "N") + ("T" if b.kstrided else "N")
        win = "w%d" % a.taps if a.taps > 1 else ("w%d" % b.taps if b.taps > 1 else "")
        desc = (f"{M}x{N}x{Kd}" + (f" b{batch}" if batch > 1 else "") + f" {lay} {DT[a.dtype]}/{DT[b.dtype]} {win}"
                + (f" sk{kw['split_k']}" if kw.get("split_k", 1) > 1 else "")
                + (" bn" if kw.get("bn_partial") is not None else "") + (" acc" if kw.get("accumulate") else "")
                + (" gelu" if kw.get("c_bf16_act") else "") + (" dgelu" if kw.get("act_grad_of") is not None else "")
                + (" colsum" if kw.get("col_sum") is not None else "") + off)
        if args.sweep and a.kstrided and b.kstrided:
            best = []
            for sk in (1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64):
                if Kd // sk < 128:
                    break
                kw2 = dict(kw, split_k=sk)
                real(M, N, Kd, a, b, c, **kw2)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(args.reps):
                    real(M, N, Kd, a, b, c, **kw2)
                e1.record()
                torch.cuda.synchronize()
                best.append((e0.elapsed_time(e1) / args.reps * 1e3, sk))
            desc += "  | " + " ".join(f"{sk}:{t:.0f}" for t, sk in best) + f"  best sk{min(best)[1]}"
        rows.append((us, fl, desc, "side" if on_side else "main"))
    tot = defaultdict(float)
    for us, fl, desc, st in sorted(rows, reverse=True):
        tot[st] += us
        print(f"{us:8.1f} us {fl / us / 1e6:7.1f} TFLOP/s  {st:4s}  {desc}")
    print(f"{len(rows)} GEMMs; main {tot['main']:.0f} us, side {tot['side']:.0f} us; "
          f"{sum(r[1] for r in rows) / 1e12:.3f} TFLOP")


if __name__ == "__main__":
    main()
