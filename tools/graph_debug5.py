"""Debug: per-parameter gradient differences between split-graph launches and single-graph
replays, repeated launches with the same inputs and no Adam."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import autoformer_amd as A  # noqa: E402
from autoformer_amd import train as TR  # noqa: E402
from autoformer_amd.detinit import det_init_, det_inputs  # noqa: E402
from autoformer_amd.layers import side_stream  # noqa: E402
from autoformer_amd.train import TrainStep  # noqa: E402
from factory.AutoVC import AutoVC  # noqa: E402

comp = sys.argv[1] if len(sys.argv) > 1 else "bf16"
B, T = (64, 128) if comp == "bf16" else (4, 64)
A.set_compute(comp)
x0, e0 = (torch.from_numpy(a).cuda() for a in det_inputs(B, T, seed=20))
res = {}
for split in (False, True):
    TR._GRAPH_SPLIT = split
    m = AutoVC(44, 256, 512, 16)
    det_init_(m)
    m = m.cuda().train()
    ts = TrainStep(m, lr=0.0)
    xb, eb = x0.clone(), e0.clone()
    ts.step(xb, eb)
    ts.capture(xb, eb, warmup=0)
    torch.cuda.synchronize()
    out = []
    for i in range(3):
        if split:
            ts.graph_split.launch(torch.cuda.current_stream(), side_stream())
        else:
            ts.graph_fb.replay()
        torch.cuda.synchronize()
        out.append({n: p.grad.clone() for n, p in m.named_parameters()})
    res[split] = out
    if split:
        print("counts", ts.graph_split.counts)
for i in range(3):
    print("launch", i, flush=True)
    for n in res[False][0]:
        a, b = res[False][0][n].double(), res[True][i][n].double()
        r = ((a - b).norm() / (a.norm() + 1e-30)).item()
        if not r < 1e-4:
            print("   ", n, f"{r:.3e}", flush=True)
