"""Debug: repeated split-graph launches without Adam in between (same inputs)."""
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
    for i in range(4):
        if split:
            ts.graph_split.launch(torch.cuda.current_stream(), side_stream())
        else:
            ts.graph_fb.replay()
        torch.cuda.synchronize()
        bad = [n for n, b in m.named_buffers() if not torch.isfinite(b).all()]
        print("split" if split else "single", i, "loss", ts.loss.item(), "gnorm", ts.gflat.norm().item(),
              "flat finite", bool(torch.isfinite(ts.flat).all()), "bad bufs", bad[:4], flush=True)
