"""Every native entry point called during one train step, grouped by (entry point, model-side call
site): count per step.  Finds the conversion / transpose / pad passes a step still makes and where
they come from.

  python tools/call_census.py [--model AutoVC|MetaConv|MetaPool] [--only avc_convert,avc_transpose_batched2]
"""
import argparse
import os
import sys
import traceback
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="MetaConv")
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    import importlib

    import autoformer_amd as A
    from autoformer_amd import _lib
    from autoformer_amd.detinit import det_init_, det_inputs
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

    only = set(s for s in args.only.split(",") if s)
    sites = Counter()
    real = _lib.call
    pkg = os.path.join("autoformer_amd", "")

    def rec(name, *a):
        if not only or name in only:
            site = "?"
            for fr in reversed(traceback.extract_stack()[:-1]):
                if pkg in fr.filename and not fr.filename.endswith(("kernels.py", "_lib.py")):
                    site = fr.filename.split(pkg)[-1] + f":{fr.lineno}"
                    break
            sites[(name, site)] += 1
        return real(name, *a)

    _lib.call = rec
    try:
        ts.step(x, e)
    finally:
        _lib.call = real
    torch.cuda.synchronize()
    print(f"# {args.model} B=64 T={T} bf16: native calls of one step by (entry point, call site)")
    for (name, site), n in sorted(sites.items(), key=lambda kv: (kv[0][0], -kv[1])):
        print(f"{n:5d}  {name:32s} {site}")
    print(f"total {sum(sites.values())}")


if __name__ == "__main__":
    main()
