"""Diagnostic: one captured MetaPool (or other) step at small batch, printing the worst ops with the
norms of kernel output vs fp64 reference (tests/capture_ref.py)."""
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import autoformer_amd as A  # noqa: E402
from autoformer_amd.detinit import det_init_  # noqa: E402
from autoformer_amd.layers import set_grad_sink  # noqa: E402
from autoformer_amd.train import TrainStep  # noqa: E402
from tests import capture_ref as CR  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "MetaPool"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
sink = (sys.argv[3] if len(sys.argv) > 3 else "1") == "1"
A.set_compute("bf16")
cls = getattr(importlib.import_module(f"autoformer_amd.factory.{name}"), name)
m = cls(44, 256, 512, 22)
det_init_(m)
m = m.cuda().train()
T = 176
g = torch.Generator().manual_seed(1234)
x = torch.clamp(torch.randn(B, T, 80, generator=g) * 1.5 - 2.5, -5.0, 2.0).cuda()
e = torch.nn.functional.normalize(torch.randn(B, 256, generator=g), dim=-1).cuda()
orig_rel = CR._rel
norms = []


def rel(got, ref, base=None):
    v = orig_rel(got, ref, base)
    gd, rd = got.double(), ref.double()
    if base is not None:
        gd, rd = gd - base, rd - base
    norms.append((v, gd.norm().item(), rd.norm().item()))
    return v


CR._rel = rel
if sink:
    ts = TrainStep(m, lr=1e-4)
    ts.step(x, e)
    torch.cuda.synchronize()
    with CR.Capture() as cap:
        ts.step(x, e)
        torch.cuda.synchronize()
    set_grad_sink(False)
else:
    with CR.Capture() as cap:
        out = m(x, e, e)
        loss = out[1].float().pow(2).mean() + out[0].float().pow(2).mean()
        loss.backward()
        torch.cuda.synchronize()
for v, op, tag, k in cap.worst()[:12]:
    print(f"{v:.3e} {tag} [{k}]")
bad = sorted(norms, key=lambda r: -r[0])[:8]
for v, gn, rn in bad:
    print(f"rel {v:.3e}  |got| {gn:.4e}  |ref| {rn:.4e}")
