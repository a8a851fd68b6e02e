"""dL/dcodes (decoder part) on the golden T128 step, fold vs unfold: where do they differ?"""
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
res = {}
for fold in (False, True):
    AV._FOLD = fold
    m = FA.AutoVC(44, 256, 512, int(g["freq"]))
    det_init_(m)
    m = m.to(DEV).train()
    x, e = torch.from_numpy(g["x"]).to(DEV), torch.from_numpy(g["emb"]).to(DEV)
    x_id, x_psnt, code = m(x, e, e)
    cap = {}
    code.register_hook(lambda gr: cap.setdefault("d", gr.detach().clone()))
    tot = F.mse_loss(x, x_id.squeeze()) + F.mse_loss(x, x_psnt.squeeze())
    m.zero_grad()
    tot.backward()
    torch.cuda.synchronize()
    res[fold] = (cap["d"].cpu().double(), x_psnt.detach().cpu().double(),
                 {n: p.grad.detach().cpu().double() for n, p in m.named_parameters()})
d0, d1 = res[False][0], res[True][0]
print("x_psnt rel diff", float((res[True][1] - res[False][1]).abs().max() / res[False][1].abs().max()))
print("dcodes rel-fro", float((d1 - d0).norm() / d0.norm()), "max abs", float((d1 - d0).abs().max()),
      "max |d0|", float(d0.abs().max()))
B, W = d0.shape
diff = (d1 - d0).abs().view(B, 8, 88)
print("per code max diff:", diff.amax(dim=(0, 2)).tolist())
print("per channel max diff (first 88):", [round(v, 9) for v in diff.amax(dim=(0, 1)).tolist()[:88]])
for n in ("encoder.lstm.weight_hh_l1_reverse", "decoder.lstm1.weight_ih_l0", "decoder.lstm1.bias_ih_l0",
          "decoder.lstm1.weight_hh_l0"):
    a, b = res[True][2][n], res[False][2][n]
    print(n, "rel-fro", float((a - b).norm() / b.norm()))
