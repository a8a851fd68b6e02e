"""Per-parameter differences after 3 bf16 TrainSteps: eager vs eager (run-to-run
nondeterminism of split-K atomics) and eager vs hipGraph replay.  Diagnostic only."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import autoformer_amd as A  # noqa: E402
from autoformer_amd.detinit import det_init_, det_inputs  # noqa: E402
from autoformer_amd.layers import set_grad_sink  # noqa: E402
from autoformer_amd.train import TrainStep  # noqa: E402
from factory.AutoVC import AutoVC  # noqa: E402

A.set_compute("bf16")
B, T = (int(v) for v in sys.argv[1:3]) if len(sys.argv) > 2 else (4, 64)


def model():
    m = AutoVC(44, 256, 512, 16)
    det_init_(m)
    return m.to("cuda:0").train()


x, e = det_inputs(B, T, seed=3)
x, e = torch.from_numpy(x).cuda(), torch.from_numpy(e).cuda()


def run(graph, steps=3):
    m = model()
    ts = TrainStep(m)
    losses = []
    if graph:
        losses.append(ts.step(x, e).item())
        ts.capture(x, e, warmup=0)
        for _ in range(steps - 1):
            losses.append(ts.step(x, e).item())
    else:
        for _ in range(steps):
            losses.append(ts.step(x, e).item())
    torch.cuda.synchronize()
    return m, losses


def diff(ma, mb, tag):
    rows = []
    for (n, pa), (_, pb) in zip(ma.named_parameters(), mb.named_parameters()):
        d = (pa - pb).abs()
        rows.append((d.max().item(), (d > 1e-5).sum().item(), n))
    rows.sort(reverse=True)
    print(f"== {tag}: {sum(r[0] > 0 for r in rows)} of {len(rows)} tensors differ")
    for r in rows[:25]:
        print(f"  {r[0]:.3e}  n>1e-5 {r[1]:7d}  {r[2]}")


try:
    ma, la = run(False)
    mb, lb = run(False)
    mc, lc = run(True)
    print("losses eager", la, "eager2", lb, "graph", lc)
    diff(ma, mb, "eager vs eager")
    diff(ma, mc, "eager vs graph")
finally:
    set_grad_sink(False)
