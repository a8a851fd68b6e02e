"""Segmented graph replay of the C2 step (graph.hip): host time of one replay's launches and the
step time, for several segment caps re-split from the same capture.

  python tools/graph_split_probe.py [steps]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from autoformer_amd import kernels as K  # noqa: E402
from autoformer_amd import set_compute  # noqa: E402
from autoformer_amd.detinit import det_init_  # noqa: E402
from autoformer_amd.factory.AutoVC import AutoVC  # noqa: E402
from autoformer_amd.train import TrainStep  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
set_compute("bf16")
dev = torch.device("cuda", 0)
m = AutoVC(44, 256, 512, 16)
det_init_(m)
m = m.to(dev).train()
x, e = bench.synthetic_batch(64, 128, 0, dev)
ts = TrainStep(m, lr=1e-4)
for _ in range(3):
    ts.step(x, e)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    ts.step(x, e)
torch.cuda.synchronize()
print(f"eager: {(time.perf_counter() - t0) / steps * 1e3:.3f} ms/step")
ts.capture(x, e)
raw = ts.graph_fb.raw_cuda_graph()
# CONFIGS: "0:<cap>" = event-ordered segments with at most <cap> segments, "1" = one main graph with
# event-record nodes (graph.hip modes)
for cfg in os.environ.get("CONFIGS", "0:4,0:8,0:64,1").split(","):
    mode, _, cap = cfg.partition(":")
    cap = int(cap or 64)
    ts.graph_split = K.GraphSplit(raw, ts._tails[0], ts._tails[1], max_segments=cap, mode=int(mode))
    for _ in range(3):
        ts.step(x, e)
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for _ in range(steps):
        h0 = time.perf_counter()
        ts.step(x, e)
        host.append(time.perf_counter() - h0)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    host.sort()
    print(f"mode {mode} max_segments {cap:3d}: {dt * 1e3:.3f} ms/step, host per step median {host[len(host) // 2] * 1e3:.3f} ms "
          f"(max {host[-1] * 1e3:.3f}), {ts.graph_split.counts}", flush=True)
ts.check()
