"""A/B of the deep-ring NT GEMM (gemm_ring.hip) against the older kernels on the C2 / C4 product
shapes, interleaved in one process (cdna_hip_programming.md §5.4 rule 24), random operands, with
an fp32 reference check of every configuration.

  python tools/ring_ab.py [--reps 20] [--rounds 3] [--only c2|c4]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import autoformer_amd as A  # noqa: E402
from autoformer_amd import _lib  # noqa: E402
from autoformer_amd import kernels as K  # noqa: E402

A.set_compute("bf16")
dev = "cuda:0"


def ring(mode, bm=0, bn=0, nst=0, gm=8, win=1):
    _lib.call("avc_gemm_set_ring", mode, bm, bn, nst, gm, win)


def ev(fn, n):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def shapes(only):
    out = []
    if only == "conv":
        return [("conv 8192x512x2560 w5", 8192, 512, 2560, dict(win=(64, 128, 512)), False),
                ("xproj 8192x4096x512", 8192, 4096, 512, {}, False)]
    if only == "bnb":  # the halo conv with / without the BN-backward reduction epilogue (avc_gemm_bnb)
        return [("conv 8192x512x2560 w5", 8192, 512, 2560, dict(win=(64, 128, 512)), False),
                ("conv 8192x512x2560 w5 bnb", 8192, 512, 2560, dict(win=(64, 128, 512)), "bnb"),
                ("conv 8192x512x2560 w5 bnb16", 8192, 512, 2560, dict(win=(64, 128, 512)), "bnb16")]
    if only == "convk":  # the halo conv at 4 / 8 / 16 / 32 channel stages: per-stage slope vs fixed cost
        return [(f"conv 8192x512x{5 * ci} w5", 8192, 512, 5 * ci, dict(win=(64, 128, ci)), False)
                for ci in (128, 256, 512, 1024)]
    if only == "utt":  # T = 176: the one-utterance halo conv (halo) vs gemm_conv.hip (halo-noutt)
        return [("conv T176 11264x512x2560 w5", 11264, 512, 2560, dict(win=(64, 176, 512)), False),
                ("conv T176 11264x512x2560 w5 bn", 11264, 512, 2560, dict(win=(64, 176, 512)), True),
                ("conv T176 11264x176x2560 w5", 11264, 176, 2560, dict(win=(64, 176, 512)), False)]
    if only in (None, "c2"):
        out += [
            ("conv 8192x512x2560 w5", 8192, 512, 2560, dict(win=(64, 128, 512)), False),
            ("conv 8192x512x2560 w5 bn", 8192, 512, 2560, dict(win=(64, 128, 512)), True),
            ("conv 8192x80x2560 w5", 8192, 80, 2560, dict(win=(64, 128, 512)), False),
            ("xproj 8192x4096x512", 8192, 4096, 512, {}, False),
            ("dx 8192x1024x4096", 8192, 1024, 4096, {}, False),
            ("dx 8192x512x4096", 8192, 512, 4096, {}, False),
            ("xproj1 8192x2048x344", 8192, 2048, 344, {}, False),
        ]
    if only in (None, "c4"):
        out += [
            ("tok1 22016x7424x1856", 22016, 7424, 1856, {}, False),
            ("tok2 22016x1849x7424", 22016, 1849, 7424, {}, False),
            ("cf1 118336x1376x344", 118336, 1376, 344, {}, False),
            ("cf2 118336x344x1376", 118336, 344, 1376, {}, False),
            ("conv T176 11264x512x2560 w5", 11264, 512, 2560, dict(win=(64, 176, 512)), False),
        ]
    return out


# (mode, bm, bn, nst, gm, win): win 2 = 5-tap convs on the halo ring kernel
CONFIGS = [("old", (0, 0, 0, 0, 0, 1)), ("auto", (-1, 0, 0, 0, 8, 1)), ("halo", (-1, 0, 0, 0, 8, 2)),
           ("128x128x4", (1, 128, 128, 4, 8, 1)), ("256x128x3", (1, 256, 128, 3, 8, 1)),
           ("256x256x2", (1, 256, 256, 2, 8, 1)), ("128x256x3", (1, 128, 256, 3, 8, 1)),
           ("auto-gm4", (-1, 0, 0, 0, 4, 1)), ("auto-gm16", (-1, 0, 0, 0, 16, 1)),
           # timing ablations of the halo conv (wrong results): its loads alone / its reads + MFMAs alone
           ("halo-loads", (-1, 0, 0, 0, 8, 3)), ("halo-math", (-1, 0, 0, 0, 8, 4)),
           ("halo-contig", (-1, 0, 0, 0, 8, 5)),
           # the warp-specialised halo conv (4 MMA waves of 64 x 64 + 4 loader waves)
           ("halo-ws", (-1, 0, 0, 0, 8, 6)),
           ("halo-mfma", (-1, 0, 0, 0, 8, 7)), ("halo-reads", (-1, 0, 0, 0, 8, 8)),
           ("halo-prio", (-1, 0, 0, 0, 8, 9)), ("halo-noutt", (-1, 0, 0, 0, 8, 10))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", default=None)
    ap.add_argument("--configs", default=None, help="comma-separated subset of the CONFIGS names")
    args = ap.parse_args()
    configs = [c for c in CONFIGS if (args.configs is None and not c[0].startswith("halo-"))
               or (args.configs is not None and c[0] in args.configs.split(","))]
    torch.manual_seed(0)
    for name, M, N, Kd, kw, bn in shapes(args.only):
        if "win" in kw:
            B, T, Ci = kw["win"]
            x = torch.randn(B * T, Ci, device=dev).bfloat16()
            opa = K.operand(x, Ci, window=(5, 2, T, T, Ci))
            # reference: explicit im2col
            xp = torch.nn.functional.pad(x.float().view(B, T, Ci), (0, 0, 2, 2))
            aref = torch.cat([xp[:, k:k + T] for k in range(5)], dim=2).reshape(B * T, 5 * Ci)
        else:
            a = torch.randn(M, Kd, device=dev).bfloat16()
            opa = K.operand(a, Kd)
            aref = a.float()
        b = (torch.randn(N, Kd, device=dev) * 0.05).bfloat16()
        c = torch.empty(M, N, device=dev)
        ref = aref @ b.float().t()
        kwb = {}
        if bn in ("bnb", "bnb16"):
            y = torch.randn(M, N, device=dev).bfloat16()
            mean, rstd = y.float().mean(0), 1 / (y.float().var(0) + 1e-5).sqrt()
            coef = torch.empty(6 * N, device=dev)
            dg, db, dbi = (torch.zeros(N, device=dev) for _ in range(3))
            kwb = dict(bnb=(y, mean, rstd, torch.ones(N, device=dev), torch.zeros(N, device=dev), K.ACT_RELU, coef,
                            dg, db, dbi, 1))
            if bn == "bnb16":
                c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        elif bn:
            part = K.bn_partial_buffer(M, N, dev)
            g_, b_ = torch.ones(N, device=dev), torch.zeros(N, device=dev)
            rm, rv = torch.zeros(N, device=dev), torch.ones(N, device=dev)
            kwb = dict(bn_partial=part, bn_fin=(g_, b_, rm, rv, None, 0.1, 1e-5, 1))

        def run():
            K.gemm(M, N, Kd, opa, K.operand(b, Kd), c, **kwb)

        res = {}
        for cname, cfg in configs:
            ring(*cfg)
            c.zero_()
            run()
            torch.cuda.synchronize()
            err = ((c - ref).abs().max() / ref.abs().max()).item()
            res[cname] = ([], err)
        for _ in range(args.rounds):
            for cname, cfg in configs:
                ring(*cfg)
                run()
                torch.cuda.synchronize()
                res[cname][0].append(ev(run, args.reps))
        fl = 2.0 * M * N * Kd
        for cname, (ts, err) in res.items():
            t = min(ts)
            print(f"{name:30s} {cname:10s} {t:8.1f} us (med {sorted(ts)[len(ts) // 2]:8.1f})  "
                  f"{fl / t / 1e6:7.1f} TF  err {err:.2e}", flush=True)
        del c, ref, aref
        torch.cuda.empty_cache()
    ring(0)


if __name__ == "__main__":
    main()
