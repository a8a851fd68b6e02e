"""Does the fold change sign(code - code_re) of the L1 code loss (its gradient) on the golden input?"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import autoformer_amd as A  # noqa: E402
import factory.AutoVC as FA  # noqa: E402
from autoformer_amd.detinit import det_init_  # noqa: E402
import autoformer_amd.factory.AutoVC as AV  # noqa: E402

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
    with torch.no_grad():
        _, x_psnt, code = m(x, e, e)
        code_re = m(x_psnt, e, None)
    d = (code - code_re).cpu().double()
    res[fold] = d
    print("fold" if fold else "nofold", "min |code-code_re| = %.3e" % d.abs().min().item(),
          "n(|d| < 1e-6) =", int((d.abs() < 1e-6).sum()), flush=True)
print("sign flips between fold and nofold:", int((torch.sign(res[True]) != torch.sign(res[False])).sum()))
print("golden sign flips vs nofold:", int((np.sign(g["codes"] - g["codes_re"]) != np.sign(res[False].numpy())).sum()),
      "vs fold:", int((np.sign(g["codes"] - g["codes_re"]) != np.sign(res[True].numpy())).sum()))
