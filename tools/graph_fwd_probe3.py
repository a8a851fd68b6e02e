"""Forward-graph diagnostic, part 3: device state outside the autograd graph that the eager
backward changes -- parameters, buffers, every PackCache value, the inputs.
python tools/graph_fwd_probe3.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def tensors_of(v):
    if isinstance(v, torch.Tensor):
        return [v]
    if isinstance(v, (tuple, list)):
        out = []
        for u in v:
            out += tensors_of(u)
        return out
    return []


def main():
    import autoformer_amd as A
    from autoformer_amd import layers as Lyr
    from autoformer_amd import train as TR
    from autoformer_amd.detinit import det_init_, det_inputs
    from autoformer_amd.factory.AutoVC import AutoVC

    A.set_compute("bf16")
    m = AutoVC(44, 256, 512, 16)
    det_init_(m)
    m = m.cuda().train()
    x, e = det_inputs(64, 128)
    x, e = torch.from_numpy(x).cuda(), torch.from_numpy(e).cuda()
    ts = TR.TrainStep(m, lr=0.0)
    try:
        ts.step(x, e)
        ts.capture(x, e, warmup=0, forward_only=True)
        ts.graph_f.replay()
        torch.cuda.synchronize()
        state = [("x", x), ("e", e)]
        state += [("param " + n, p) for n, p in m.named_parameters()]
        state += [("buffer " + n, b) for n, b in m.named_buffers()]
        for i, ref in enumerate(Lyr._PLAN):
            c = ref()
            if c is not None:
                state += [(f"pack {i}[{j}]", t) for j, t in enumerate(tensors_of(c.val))]
        snap = [(n, t, t.detach().clone()) for n, t in state]
        print(f"{len(snap)} tensors watched", flush=True)
        ts.gflat.zero_()
        ts.loss.backward(retain_graph=True)
        Lyr.join_side()
        torch.cuda.synchronize()
        for n, t, r in snap:
            if not torch.equal(t.detach(), r):
                print("changed by the backward:", n, tuple(t.shape), t.dtype, flush=True)
        print("done", flush=True)
    finally:
        Lyr.set_grad_sink(False)


if __name__ == "__main__":
    main()
