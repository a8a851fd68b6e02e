"""The step replayed as captured hipGraphs (TrainStep.capture: the segmented main / side replay, one
graph, the forward-only graph) against the eager step.

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


def _compare(comp, B, T, freq, gtol, steps=4, forward_only=False, split=None, lr=0.0, ptol=None):
    from autoformer_amd.detinit import det_inputs
    from autoformer_amd.layers import set_grad_sink
    from autoformer_amd.train import TrainStep

    batches = [tuple(torch.from_numpy(a).to(DEV) for a in det_inputs(B, T, seed=20 + i)) for i in range(steps)]
    ma, mb = _model(comp, freq), _model(comp, freq)
    ta, tb = TrainStep(ma, lr=lr), TrainStep(mb, lr=lr)
    xb, eb = batches[0][0].clone(), batches[0][1].clone()
    try:
        if lr:
            # same starting point: one eager step on each (the capture itself runs no step)
            ta.step(xb, eb)
        tb.step(xb, eb)
        tb.capture(xb, eb, warmup=0, forward_only=forward_only, split=split)
        if forward_only:
            assert tb.graph_f is not None
        elif split is False:
            assert tb.graph_fb is not None and tb.graph_split is None
        else:
            assert tb.graph_split is not None, "the default capture is the segmented main / side replay"
            c = tb.graph_split.counts
            assert c["side_nodes"] > 0 and c["cross_edges"] > 0, c
            assert c["segments"] > 1, c
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
            assert torch.isfinite(lb).item(), (i, lb.item())
            assert abs(la.item() - lb.item()) <= 1e-4 * abs(la.item()), (i, la.item(), lb.item())
            for (n, pa), (_, pb) in zip(ma.named_parameters(), mb.named_parameters()):
                a, b = pa.grad.double(), pb.grad.double()
                assert (a - b).norm() <= gtol * a.norm() + 1e-6, (i, n, ((a - b).norm() / a.norm()).item())
                if ptol is not None:
                    a, b = pa.detach().double(), pb.detach().double()
                    assert (a - b).norm() <= ptol * a.norm() + 1e-8, (i, n, ((a - b).norm() / a.norm()).item())
            del ga
        tb.check()
    finally:
        set_grad_sink(False)


def test_graph_replay_matches_eager_fp32():
    """The one-graph form (split=False)."""
    _compare("fp32", 4, 64, 16, 1e-4, split=False)


def test_graph_replay_matches_eager_bf16_c2():
    """At the C2 shape (B=64, T=128, bf16: the persistent recurrences, split-K weight gradients,
    halo conv kernels), one graph.  bf16 run-to-run spread of a gradient tensor is ~1e-3 (split-K order)."""
    _compare("bf16", 64, 128, 16, 1e-2, split=False)


def test_split_graph_replay_matches_eager_fp32():
    """The segmented main / side replay (graph.hip): 10 replays, new batch each, lr = 0."""
    _compare("fp32", 4, 64, 16, 1e-4, steps=10)


def test_split_graph_replay_matches_eager_bf16_c2():
    """The segmented main / side replay at the C2 shape over 10 replays: any
    side-stream weight-gradient node that ran before the main node it depends on, or a replay that
    read the previous replay's flags / accumulators, shows as an O(1) gradient error or NaN."""
    _compare("bf16", 64, 128, 16, 1e-2, steps=10)


def test_split_graph_replay_trains_like_eager_fp32():
    """lr > 0 over 10 replays (Adam inside the graph): every replay's forward must see the weights
    and packs the previous replay's optimizer step produced (parameters compared too)."""
    _compare("fp32", 4, 64, 16, 1e-3, steps=10, lr=1e-3, ptol=1e-4)


def test_forward_graph_matches_eager_fp32():
    """capture(forward_only=True): forward replayed, backward eager over the retained graph."""
    _compare("fp32", 4, 64, 16, 1e-4, forward_only=True)


def test_forward_graph_matches_eager_bf16_c2():
    _compare("bf16", 64, 128, 16, 1e-2, forward_only=True)


def test_forward_graph_trains_like_eager_fp32():
    """lr > 0 over several steps with the forward graph: each step's eager backward must
    see the packs of the current weights, not a stale pack from the captured forward."""
    _compare("fp32", 4, 64, 16, 1e-3, steps=5, forward_only=True, lr=1e-3, ptol=1e-4)
