"""Debug: split-graph replays with a new batch each replay; loss finiteness + fault word."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import autoformer_amd as A  # noqa: E402
from autoformer_amd import kernels as K  # noqa: E402
from autoformer_amd.detinit import det_init_, det_inputs  # noqa: E402
from autoformer_amd.train import TrainStep  # noqa: E402
from factory.AutoVC import AutoVC  # noqa: E402

comp = sys.argv[1] if len(sys.argv) > 1 else "bf16"
B, T = (64, 128) if comp == "bf16" else (4, 64)
A.set_compute(comp)
m = AutoVC(44, 256, 512, 16)
det_init_(m)
m = m.cuda().train()
batches = [tuple(torch.from_numpy(a).cuda() for a in det_inputs(B, T, seed=20 + i)) for i in range(6)]
ts = TrainStep(m, lr=0.0)
xb, eb = batches[0][0].clone(), batches[0][1].clone()
ts.step(xb, eb)
ts.capture(xb, eb, warmup=0)
print("split", None if ts.graph_split is None else ts.graph_split.counts, flush=True)
for i, (x, e) in enumerate(batches):
    xb.copy_(x)
    eb.copy_(e)
    loss = ts.step(xb, eb)
    torch.cuda.synchronize()
    fw = int(K.fault_word().item())
    g = ts.gflat
    print(i, "loss", loss.item(), "fault", fw, "grad finite", bool(torch.isfinite(g).all()), "gnorm", g.norm().item(),
          flush=True)
