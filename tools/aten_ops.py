"""Which ATen / runtime GPU operations remain in the AutoVC C2 train step, and where the Python
code issues them (torch.profiler, one step after warm-up, stacks trimmed to autoformer_amd).

  python tools/aten_ops.py
"""
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    import autoformer_amd as A
    from autoformer_amd.detinit import det_init_, det_inputs
    from autoformer_amd.factory.AutoVC import AutoVC
    from autoformer_amd.train import TrainStep

    A.set_compute("bf16")
    m = AutoVC(44, 256, 512, 16)
    det_init_(m)
    m = m.cuda().train()
    x, e = det_inputs(64, 128)
    x, e = torch.from_numpy(x).cuda(), torch.from_numpy(e).cuda()
    ts = TrainStep(m)
    for _ in range(3):
        ts.step(x, e)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
        ts.step(x, e)
        torch.cuda.synchronize()
    keep = ("aten::copy_", "aten::fill_", "aten::zero_", "aten::add", "aten::add_", "aten::mul", "aten::sum",
            "aten::cat", "aten::clone", "aten::contiguous", "aten::sub", "aten::div", "aten::mean", "aten::neg",
            "aten::zeros", "aten::zeros_like", "aten::ones_like", "aten::full", "aten::to", "aten::_to_copy",
            "aten::abs", "aten::pow", "aten::mse_loss", "aten::l1_loss", "aten::expand", "aten::index")
    agg = defaultdict(int)
    for ev in prof.events():
        if ev.name not in keep or ev.cpu_parent is not None and ev.cpu_parent.name in keep:
            continue
        st = [s for s in (ev.stack or []) if "autoformer_amd" in s or "torch/autograd" in s]
        where = " <- ".join(s.split("autoformer_amd/")[-1] for s in st[:3]) or "(no python frame)"
        agg[(ev.name, str(ev.input_shapes)[:60], where)] += 1
    for (name, shp, where), n in sorted(agg.items(), key=lambda kv: -kv[1]):
        print(f"{n:3d}  {name:18s} {shp:60s} {where}")


if __name__ == "__main__":
    main()
