"""Algorithmic FLOPs per mel-frame of one training step for the model variants, counted the
way SURVEY.md §8(d) counted AutoVC: torch.utils.flop_counter over the *reference* modules on
the CPU with oneDNN disabled (so nn.LSTM lowers to counted matmuls).  Survey container only
(imports /root/reference); the numbers are copied into bench.py's FLOP_PER_FRAME.

    PYTHONDONTWRITEBYTECODE=1 python tools/variant_flops.py
"""
import sys

import torch
import torch.nn.functional as F
from torch.utils.flop_counter import FlopCounterMode

sys.dont_write_bytecode = True
sys.path.insert(0, "/root/reference")
torch.manual_seed(0)


def step_flops(name, T, freq, B=2):
    mod = __import__(f"factory.{name}", fromlist=[name])
    cls = getattr(mod, name, None) or getattr(mod, name.split("_")[0])
    m = cls(44, 256, 512, freq).train()
    x = torch.randn(B, T, 80)
    e = F.normalize(torch.randn(B, 256), dim=-1)
    with torch.backends.mkldnn.flags(enabled=False), FlopCounterMode(display=False) as fc:
        out = m(x, e, e)
        if name.endswith("_Adjust"):
            emb_adj, out = out[0], out[1:]
        loss = F.mse_loss(x, out[0].squeeze()) + F.mse_loss(x, out[1].squeeze())
        re = m(out[1], e, None)
        re = re[0] if isinstance(re, tuple) else re
        loss = loss + F.l1_loss(out[2], re)
        if name.endswith("_Adjust"):
            loss = loss + F.l1_loss(emb_adj, e)
        loss.backward()
    return fc.get_total_flops() / (B * T)


if __name__ == "__main__":
    cases = [("AutoVC", 128, 16), ("AutoVC2", 128, 16), ("AutoVC_Adjust", 128, 16), ("AutoVC2", 176, 22),
             ("AutoVC_Adjust", 176, 22), ("MetaConv2", 176, 22), ("MetaPool2", 176, 22),
             ("MetaConv_Adjust", 176, 22), ("MetaPool_Adjust", 176, 22)]
    for n, T, f in cases:
        print(f"{n:16s} T={T} freq={f}: {step_flops(n, T, f) / 1e6:.2f} MFLOP/frame", flush=True)
