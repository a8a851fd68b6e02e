"""Sensitivity of the encoder gradient heads (golden T128 step, fp32) to a 1e-6 relative
perturbation of dL/dcodes: the margin of the fp32 golden check for each tensor, unperturbed and
perturbed (unfolded decoder path)."""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import autoformer_amd as A  # noqa: E402
import autoformer_amd.factory.AutoVC as AV  # noqa: E402
import factory.AutoVC as FA  # noqa: E402
from autoformer_amd.detinit import det_init_  # noqa: E402

DEV = "cuda:0"
g = np.load(os.path.join(ROOT, "tests", "golden", "autovc_T128.npz"))
A.set_compute("fp32")
AV._FOLD = False
grads = {}
for eps in (0.0, 1e-6, 1e-7):
    m = FA.AutoVC(44, 256, 512, int(g["freq"]))
    det_init_(m)
    m = m.to(DEV).train()
    x, e = torch.from_numpy(g["x"]).to(DEV), torch.from_numpy(g["emb"]).to(DEV)
    x_id, x_psnt, code = m(x, e, e)
    gen = torch.Generator(device=DEV).manual_seed(1)
    if eps:
        code.register_hook(lambda gr: gr * (1 + eps * torch.randn(gr.shape, device=DEV, generator=gen)))
    tot = F.mse_loss(x, x_id.squeeze()) + F.mse_loss(x, x_psnt.squeeze()) + F.l1_loss(code, m(x_psnt, e, None))
    m.zero_grad()
    tot.backward()
    torch.cuda.synchronize()
    grads[eps] = {n: p.grad.detach().cpu().double().reshape(-1) for n, p in m.named_parameters()}
for eps in (1e-6, 1e-7):
    rows = []
    for n in grads[0.0]:
        head = g["ghead/" + n].astype(np.float64)
        d = (grads[eps][n][:64] - grads[0.0][n][:64]).abs().max().item()
        rows.append((d / max(1e-2 * np.abs(head).max(), 1e-6), n, d))
    rows.sort(reverse=True)
    print("perturbation %.0e of dL/dcodes -> head change / bar:" % eps)
    for r in rows[:5]:
        print("  %.3f  %-45s %.3e" % r)
