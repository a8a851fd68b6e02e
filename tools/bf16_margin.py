"""bf16 golden margins of tests/test_gpu_model.py::test_autovc_bf16_loose: rel-inf of mel_postnet
and the losses against the reference goldens (A/B of code-path switches via the environment)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.test_gpu_model import _model, _step  # noqa: E402
from tests.helpers import rel_inf  # noqa: E402

for fname in ("autovc_T128.npz", "autovc_T176.npz"):
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", fname)))
    m = _model(int(g["freq"]), "bf16")
    x, e = torch.from_numpy(g["x"]).to("cuda:0"), torch.from_numpy(g["emb"]).to("cuda:0")
    outs, losses, total = _step(m, x, e)
    torch.cuda.synchronize()
    r = [rel_inf(o.detach().cpu(), g[k]) for o, k in zip(outs[:2], ("mel", "mel_psnt"))]
    rf = [float(np.linalg.norm(o.detach().cpu().numpy().ravel() - g[k].ravel()) / np.linalg.norm(g[k].ravel()))
          for o, k in zip(outs[:2], ("mel", "mel_psnt"))]
    lr = np.abs(np.array([l.item() for l in losses]) / g["losses"] - 1).max()
    print(f"{fname} bf16: mel rel-inf {r[0]:.3e} rel-frob {rf[0]:.3e}, mel_psnt rel-inf {r[1]:.3e} rel-frob "
          f"{rf[1]:.3e}, losses rel {lr:.2e}", flush=True)
