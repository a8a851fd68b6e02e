"""MetaPool fp32 golden step: per-parameter gradient-head error (scaled as tests/helpers.py's
grad_mismatches does) with the one-pass LayerNorm backward on and off, to bisect which form moves
decoder.output_conv_2.1.bias.

  python tools/metapool_head_probe.py [metapool|metaconv]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import autoformer_amd as A  # noqa: E402
from autoformer_amd import kernels as K  # noqa: E402
from autoformer_amd.detinit import det_init_  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "metapool"
g = np.load(os.path.join(ROOT, "tests", "golden", f"{kind}_T176.npz"))
DEV = "cuda:0"


def run(label):
    A.set_compute("fp32")
    if kind == "metaconv":
        from factory.MetaConv import MetaConv as M
    else:
        from factory.MetaPool import MetaPool as M
    m = M(44, 256, 512, 22)
    det_init_(m)
    m = m.to(DEV).train()
    x, e = (torch.from_numpy(g[k]).to(DEV) for k in ("x", "emb"))
    x_id, x_psnt, code = m(x, e, e)
    l1 = F.mse_loss(x, x_id.squeeze())
    l2 = F.mse_loss(x, x_psnt.squeeze())
    code_re = m(x_psnt, e, None)
    l3 = F.l1_loss(code, code_re)
    m.zero_grad()
    (l1 + l2 + l3).backward()
    torch.cuda.synchronize()
    rows = []
    for name, p in m.named_parameters():
        ref_n = float(g["gnorm/" + name])
        got = p.grad.detach().cpu().double()
        head = g["ghead/" + name].astype(np.float64)
        err = np.abs(got.reshape(-1)[:64].numpy() - head).max()
        scale = max(np.abs(head).max(), ref_n / np.sqrt(max(p.numel(), 1)), 1e-6)
        rows.append((err / scale, abs(got.norm().item() - ref_n) / max(ref_n, 1e-12), name))
    rows.sort(reverse=True)
    print(f"== {label}: losses {[round(v.item(), 7) for v in (l1, l2, l3)]} golden {g['losses'].tolist()}")
    for r in rows:
        if "output_conv_2.1.bias" in r[2]:
            print(f"   head {r[0]:.4f}  norm {r[1]:.2e}  {r[2]}  (VERDICT r4 item 3)")
    for r in rows[:6]:
        print(f"   head {r[0]:.4f}  norm {r[1]:.2e}  {r[2]}")


for rep in range(int(os.environ.get("REPS", "1"))):
    run(f"default #{rep}")
orig = K.ln_vec
K.ln_vec = lambda D: False
try:
    run("two-pass LayerNorm backward (ln_vec off)")
finally:
    K.ln_vec = orig
run("default again")
