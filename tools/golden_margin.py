"""Per-parameter margins of the fp32 golden gradient check (tests/test_gpu_model.py): err / bar
for the gradient heads, to see how close each tensor is to its bar (AVC_FOLD=0/1 A/B)."""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import autoformer_amd as A  # noqa: E402
from autoformer_amd.detinit import det_init_  # noqa: E402
from factory.AutoVC import AutoVC  # noqa: E402

DEV = "cuda:0"
for fname in ("autovc_T128.npz", "autovc_T176.npz"):
    g = np.load(os.path.join(ROOT, "tests", "golden", fname))
    A.set_compute("fp32")
    m = AutoVC(44, 256, 512, int(g["freq"]))
    det_init_(m)
    m = m.to(DEV).train()
    x, e = torch.from_numpy(g["x"]).to(DEV), torch.from_numpy(g["emb"]).to(DEV)
    x_id, x_psnt, code = m(x, e, e)
    tot = F.mse_loss(x, x_id.squeeze()) + F.mse_loss(x, x_psnt.squeeze()) + F.l1_loss(code, m(x_psnt, e, None))
    m.zero_grad()
    tot.backward()
    torch.cuda.synchronize()
    rows = []
    for name, p in m.named_parameters():
        head = g["ghead/" + name].astype(np.float64)
        got = p.grad.detach().cpu().double().reshape(-1)[:64].numpy()
        err = np.abs(got - head).max()
        rows.append((err / max(1e-2 * np.abs(head).max(), 1e-6), name, err, np.abs(head).max()))
    rows.sort(reverse=True)
    print(fname, "fold" if os.environ.get("AVC_FOLD", "1") != "0" else "nofold")
    for r in rows[:8]:
        print("  %.3f  %-45s err %.3e  headmax %.3e" % r)
