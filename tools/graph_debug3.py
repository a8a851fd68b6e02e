"""Debug: optimizer / flat-buffer state after one split-graph replay vs the single graph."""
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
res = []
for split in (False, True):
    TR._GRAPH_SPLIT = split
    m = AutoVC(44, 256, 512, 16)
    det_init_(m)
    m = m.cuda().train()
    ts = TrainStep(m, lr=0.0)
    xb, eb = x0.clone(), e0.clone()
    ts.step(xb, eb)
    torch.cuda.synchronize()
    st0 = ts.opt.state.clone()
    ts.capture(xb, eb, warmup=0)
    torch.cuda.synchronize()
    st1 = ts.opt.state.clone()
    loss = ts.step(xb, eb)
    torch.cuda.synchronize()
    d = dict(loss=loss.item(), state0=st0.tolist(), state_cap=st1.tolist(), state=ts.opt.state.tolist())
    for k, t in (("flat", ts.flat), ("gflat", ts.gflat), ("m", ts.opt.m), ("v", ts.opt.v)):
        fin = torch.isfinite(t)
        d[k] = (int((~fin).sum()), float(t[fin].double().norm()))
    print("split" if split else "single", d, flush=True)
