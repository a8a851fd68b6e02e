"""The recorded step (TrainStep.record, autoformer_amd/replay.py) replayed against the eager step.

Both trainers start from the same weights (deterministic mode: no split-K float atomics, so two eager
runs agree to the last bit, tools/eager_pair.py) and take one eager step; then one records its next step
while the other steps eagerly, and every later step is a replay of the record against an eager step
on the same NEW batch.  With lr > 0 every replay must see the weights, Adam moments and weight packs
the previous replay produced (parameters compared after every step), and a kernel whose recorded
arguments pointed at memory the replay no longer owns, or a side-stream kernel that lost its event
edge, shows as an O(1) gradient error or NaN."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
# torch ops of the recorded AutoVC step: the gradient buffer's zero fill and autograd's sums of the
# gradients of tensors with two consumers (replayed through aten.add.out into the recorded tensor)
_OPS = ["aten.zero_.default", "aten.add.Tensor"]


def _autovc(comp, freq):
    import autoformer_amd as A
    from autoformer_amd.detinit import det_init_
    from factory.AutoVC import AutoVC

    A.set_compute(comp)
    m = AutoVC(44, 256, 512, freq)
    det_init_(m)
    return m.to(DEV).train()


def _compare(make, B, T, gtol=0.0, steps=6, lr=1e-4, ptol=0.0, torch_ops=None):
    from autoformer_amd.detinit import det_inputs
    from autoformer_amd.layers import set_grad_sink
    from autoformer_amd.train import TrainStep

    import autoformer_amd.kernels as K

    batches = [tuple(torch.from_numpy(a).to(DEV) for a in det_inputs(B, T, seed=40 + i)) for i in range(steps)]
    (ma, ta), (mb, tb) = make(lr), make(lr)
    # no split-K: the weight gradients are not sums of float atomics in arrival order, so two runs of
    # the same kernels agree to the last bit -- Adam's first steps (update ~ lr * sign(g)) would
    # otherwise amplify the bf16 split-K order noise of near-zero gradient elements
    K.set_deterministic(True)
    try:
        ta.step(*batches[0])
        tb.step(*batches[0])
        xb, eb = batches[1][0].clone(), batches[1][1].clone()
        for i, (x, e) in enumerate(batches[1:], 1):
            la = ta.step(x, e)
            if i == 1:
                rec = tb.record(xb, eb, warmup=0)
                lb = tb.loss
                assert rec.native_calls() > 50, rec.native_calls()
                if torch_ops is not None:
                    assert sorted(set(rec.torch_ops)) == sorted(torch_ops), rec.torch_ops
            else:
                lb = tb.step(x, e)  # copied into the recorded input tensors
            torch.cuda.synchronize()
            assert torch.isfinite(lb).item(), (i, lb.item())
            assert abs(la.item() - lb.item()) <= gtol * abs(la.item()), (i, la.item(), lb.item())
            bad = []
            for (n, pa), (_, pb) in zip(ma.named_parameters(), mb.named_parameters()):
                a, b = pa.grad.double(), pb.grad.double()
                if (a - b).norm() > gtol * a.norm():
                    bad.append(("grad", n, ((a - b).norm() / a.norm()).item()))
                if ptol is not None:
                    a, b = pa.detach().double(), pb.detach().double()
                    if (a - b).norm() > ptol * a.norm():
                        bad.append(("param", n, ((a - b).norm() / a.norm()).item()))
            assert not bad, (i, len(bad), sorted(bad, key=lambda r: -r[2])[:6])
        tb.check()
    finally:
        K.set_deterministic(False)
        set_grad_sink(False)


def _autovc_trainer(comp, freq):
    from autoformer_amd.train import TrainStep

    def make(lr):
        m = _autovc(comp, freq)
        return m, TrainStep(m, lr=lr)
    return make


def test_replay_trains_like_eager_fp32():
    """fp32 mode, lr > 0 over 5 replays: gradients, loss and parameters after every step bit-identical
    to the eager step's (deterministic mode: the replay runs the same kernels on the same values)."""
    _compare(_autovc_trainer("fp32", 16), 4, 64, lr=1e-3, torch_ops=_OPS)


def test_replay_trains_like_eager_bf16_c2():
    """The C2 shape (B=64, T=128, bf16): the persistent recurrences, the split-K weight gradients on the
    side stream, the fused BN-backward halo convs, the decoder-slice Adam + repack on the side
    stream."""
    _compare(_autovc_trainer("bf16", 16), 64, 128, steps=8, torch_ops=_OPS)


def test_replay_gan_step_bf16():
    """The two-model step (AutoVC + Discriminator, train_with_discriminator.py) recorded: its extra
    loss term is a torch add, replayed as a closure into the recorded tensor."""
    import autoformer_amd as A
    from autoformer_amd.detinit import det_init_
    from autoformer_amd.factory.Discriminator import Discriminator
    from autoformer_amd.train import TrainStep, gan_extra

    def make(lr):
        A.set_compute("bf16")
        m = _autovc("bf16", 22)
        d = Discriminator(crop_len=176)
        det_init_(d)
        d = d.to(DEV).train()
        return m, TrainStep(m, lr=lr, extra=gan_extra(d), extra_modules=[d])
    _compare(make, 8, 176, steps=4)


def test_replay_metaconv_fp32():
    """A MetaFormer family (MetaConv, T=176) recorded and replayed."""
    import autoformer_amd as A
    from autoformer_amd.detinit import det_init_
    from autoformer_amd.train import TrainStep
    from factory.MetaConv import MetaConv

    def make(lr):
        A.set_compute("fp32")
        m = MetaConv(44, 256, 512, 22)
        det_init_(m)
        m = m.to(DEV).train()
        return m, TrainStep(m, lr=lr)
    _compare(make, 2, 176, steps=4, lr=1e-3)
