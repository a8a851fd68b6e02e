"""Chaos floor of the MetaFormer fp32 golden gradients: the CPU oracle's step with every LayerNorm /
GroupNorm output perturbed by ~1 ulp of relative noise (a different fp32 summation order), N seeds.
ReLU / activation decisions of values near 0 flip, and the gradient heads of the BatchNorm layers
after them move by whole-element amounts; prints, per model, the largest head deviation from the
golden (relative to the tensor's scale, as tests/helpers.grad_mismatches measures it).

  python tools/flip_spread.py [N]
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import autovc_cpu as A  # noqa: E402
from oracle import metaformer_cpu as M  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    gen = torch.Generator().manual_seed(0)
    ln0, gn0 = F.layer_norm, F.group_norm

    def noisy(fn):
        def f(x, *a, **k):
            y = fn(x, *a, **k)
            return y * (1 + 6e-8 * torch.randn(y.shape, generator=gen, dtype=y.dtype))
        return f

    F.layer_norm, F.group_norm = noisy(ln0), noisy(gn0)
    for kind, spec, fwd in (("metaconv", M.metaconv_spec, M.metaconv_forward),
                            ("metapool", M.metapool_spec, M.metapool_forward)):
        g = np.load(os.path.join(ROOT, "tests", "golden", f"{kind}_T176.npz"))
        worst = {}
        for _ in range(n):
            sd = A.make_state(spec())
            x, e = torch.from_numpy(g["x"]), torch.from_numpy(g["emb"])
            _, tot, _ = A.step_losses(lambda a, b, c: fwd(sd, a, b, c, dim_neck=44, freq=int(g["freq"])), x, e)
            tot.backward()
            for k, t in sd.items():
                if not t.requires_grad or "conv.bias" in k or (kind == "metapool" and k.endswith("norm1.bias")):
                    continue
                hg = g["ghead/" + k].astype(np.float64)
                sc = max(np.abs(hg).max(), float(g["gnorm/" + k]) / np.sqrt(t.numel()), 1e-6)
                d = np.abs(t.grad.reshape(-1)[:64].double().numpy() - hg).max() / sc
                worst[k] = max(worst.get(k, 0.0), d)
        top = sorted(((v, k) for k, v in worst.items()), reverse=True)[:6]
        print(f"{kind}: {n} perturbed fp32 oracle steps, largest head deviation / scale: "
              + ", ".join(f"{k} {v:.3f}" for v, k in top))


if __name__ == "__main__":
    main()
