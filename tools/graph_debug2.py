"""Debug: per-parameter gradients of split-graph replay 0 vs the single-graph replay 0."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import autoformer_amd as A  # noqa: E402
from autoformer_amd import train as TR  # noqa: E402
from autoformer_amd.detinit import det_init_, det_inputs  # noqa: E402
from autoformer_amd.train import TrainStep  # noqa: E402
from factory.AutoVC import AutoVC  # noqa: E402

comp = sys.argv[1] if len(sys.argv) > 1 else "bf16"
B, T = (64, 128) if comp == "bf16" else (4, 64)
A.set_compute(comp)
x0, e0 = (torch.from_numpy(a).cuda() for a in det_inputs(B, T, seed=20))
x1, e1 = (torch.from_numpy(a).cuda() for a in det_inputs(B, T, seed=21))
res = []
for split in (False, True):
    TR._GRAPH_SPLIT = split
    m = AutoVC(44, 256, 512, 16)
    det_init_(m)
    m = m.cuda().train()
    ts = TrainStep(m, lr=0.0)
    xb, eb = x0.clone(), e0.clone()
    ts.step(xb, eb)
    ts.capture(xb, eb, warmup=0)
    xb.copy_(x1)
    eb.copy_(e1)
    out = []
    for i in range(2):
        loss = ts.step(xb, eb)
        torch.cuda.synchronize()
        out.append((loss.item(), {n: p.grad.clone() for n, p in m.named_parameters()},
                    {n: b.clone() for n, b in m.named_buffers()}, {n: p.detach().clone() for n, p in m.named_parameters()}))
    res.append(out)
for i in range(2):
    print("replay", i, "loss single", res[0][i][0], "split", res[1][i][0], flush=True)
    for n in res[0][i][1]:
        a, b = res[0][i][1][n].double(), res[1][i][1][n].double()
        r = ((a - b).norm() / (a.norm() + 1e-30)).item()
        if not r < 1e-2:
            print("  grad", n, r, flush=True)
    for n in res[0][i][2]:
        a, b = res[0][i][2][n].double(), res[1][i][2][n].double()
        r = ((a - b).norm() / (a.norm() + 1e-30)).item()
        if not r < 1e-3:
            print("  buf", n, r, flush=True)
    for n in res[0][i][3]:
        a, b = res[0][i][3][n].double(), res[1][i][3][n].double()
        if not torch.equal(a, b):
            print("  param", n, ((a - b).norm() / (a.norm() + 1e-30)).item(), flush=True)
