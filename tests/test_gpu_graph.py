"""The step replayed as a captured hipGraph (TrainStep.capture: one graph) against the eager
step.

Each replay gets a NEW batch (copied into the captured input tensors) and lr = 0, so a weight-gradient
kernel that ran before the node it depends on would read the previous batch's
activations / data gradients and show as an O(1) gradient error, while rounding differences stay
tiny (fp32: the split-K weight gradients add in a run-dependent order)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _model(comp, freq):
    import autoformer_amd as A
    from autoformer_amd.detinit import det_init_
    from factory.AutoVC import AutoVC

    A.set_compute(comp)
    m = AutoVC(44, 256, 512, freq)
    det_init_(m)
    return m.to(DEV).train()


def _compare(comp, B, T, freq, gtol, steps=4, forward_only=False):
    from autoformer_amd.detinit import det_inputs
    from autoformer_amd.layers import set_grad_sink
    from autoformer_amd.train import TrainStep

    batches = [tuple(torch.from_numpy(a).to(DEV) for a in det_inputs(B, T, seed=20 + i)) for i in range(steps)]
    ma, mb = _model(comp, freq), _model(comp, freq)
    ta, tb = TrainStep(ma, lr=0.0), TrainStep(mb, lr=0.0)
    xb, eb = batches[0][0].clone(), batches[0][1].clone()
    try:
        tb.step(xb, eb)
        tb.capture(xb, eb, warmup=0, forward_only=forward_only)
        assert (tb.graph_f if forward_only else tb.graph_fb) is not None
        for i, (x, e) in enumerate(batches):
            la = ta.step(x, e)
            ga = ta.gflat.clone()
            if forward_only:
                lb = tb.step(x, e)  # copied into the capture-time inputs by step() (through .data)
            else:
                xb.copy_(x)
                eb.copy_(e)
                lb = tb.step(xb, eb)
            torch.cuda.synchronize()
            gb = tb.gflat.clone()
            assert abs(la.item() - lb.item()) <= 1e-4 * abs(la.item()), (i, la.item(), lb.item())
            for (n, pa), (_, pb) in zip(ma.named_parameters(), mb.named_parameters()):
                a, b = pa.grad.double(), pb.grad.double()
                assert (a - b).norm() <= gtol * a.norm() + 1e-6, (i, n, ((a - b).norm() / a.norm()).item())
        tb.check()
    finally:
        set_grad_sink(False)


def test_graph_replay_matches_eager_fp32():
    _compare("fp32", 4, 64, 16, 1e-4)


def test_graph_replay_matches_eager_bf16_c2():
    """At the C2 shape (B=64, T=128, bf16: the persistent recurrences, split-K weight gradients,
    halo conv kernels).  bf16 run-to-run spread of a gradient tensor is ~1e-3 (split-K order)."""
    _compare("bf16", 64, 128, 16, 1e-2)


def test_forward_graph_matches_eager_fp32():
    """capture(forward_only=True): forward replayed, backward eager over the retained graph."""
    _compare("fp32", 4, 64, 16, 1e-4, forward_only=True)


def test_forward_graph_matches_eager_bf16_c2():
    _compare("bf16", 64, 128, 16, 1e-2, forward_only=True)
