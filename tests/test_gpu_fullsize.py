"""Full-size checks of the production (bf16) step at BASELINE.json's configurations
(SURVEY.md §8(d)): C2 AutoVC B=64 T=128 freq=16; C4 MetaConv B=64 T=176 freq=22; C5 AutoVC +
Discriminator B=64 T=176 freq=22.

The fp32 goldens pin the math at small batch; here the bf16 kernels at full size (persistent
recurrences at 256 workgroups, split-K GEMMs, halo convolutions) are held to the fp32 HIP
step on the SAME weights and inputs:
  * mel_postnet rel-inf <= 5e-2 (the bf16 bar of SURVEY §8(c): bf16 autocast on the reference
    itself sits at 3.6e-2),
  * each parameter gradient within rel-Frobenius max(GRAD_BAR, SENS_FACTOR x s) of the fp32
    one, where s is the same tensor's movement when the fp32 step runs on bf16-rounded
    weights (the gradient's own sensitivity to the rounding bf16 compute starts from);
    BN-fed conv biases, whose true gradient is 0, only finite.  The deviation grows along the backward chain: C2
    measured a median of 0.06 and at most 0.14 on the encoder, whose gradients pass through
    the decoder's three LSTM layers (bf16 operands and hand-offs) over 128 steps.  (bf16
    autocast on the reference itself is no bar here: on CPU it moves these gradients by ~100 %.)
  * losses finite and decreasing over three TrainStep steps on a fixed batch.
"""
import numpy as np
import pytest
import torch

from tests.helpers import rel_inf

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
GRAD_BAR = 0.2  # C2 measured: median 0.06, worst 0.143 (encoder BN bias: the longest backward chain)
SENS_FACTOR = 3.0


def _synthetic(B, T, seed=0):
    g = torch.Generator().manual_seed(1234 + seed)
    x = torch.clamp(torch.randn(B, T, 80, generator=g) * 1.5 - 2.5, -5.0, 2.0)
    g2 = torch.Generator().manual_seed(5678 + seed)
    e = torch.nn.functional.normalize(torch.randn(B, 256, generator=g2), dim=-1)
    return x.to(DEV), e.to(DEV)


def _bn_fed_bias(name):
    # every AutoVC / MetaFormer ConvNorm feeds a training-mode BatchNorm: its bias gradient is
    # analytically zero and both computations return rounding noise
    return "conv.bias" in name


def _fwd_bwd(model, x, e, extra=None):
    from autoformer_amd.train import losses_for

    for p in model.parameters():
        p.grad = None
    loss, parts, x_psnt = losses_for(model)(model, x, e)
    if extra is not None:
        for p in extra.parameters():
            p.grad = None
        loss = loss + extra_loss(extra, x, x_psnt)
    loss.backward()
    torch.cuda.synchronize()
    grads = {n: p.grad.detach().clone() for n, p in model.named_parameters()}
    if extra is not None:
        grads.update({"D." + n: p.grad.detach().clone() for n, p in extra.named_parameters()})
    return loss.item(), x_psnt.detach().clone(), grads


def extra_loss(D, x, x_psnt):
    from autoformer_amd.train import discriminator_loss
    return discriminator_loss(D(x), D(x_psnt.squeeze()))


def _check(name, freq, B, T, disc=False):
    import importlib

    import autoformer_amd as A
    from autoformer_amd.detinit import det_init_
    from autoformer_amd.layers import set_grad_sink
    from autoformer_amd.train import TrainStep, gan_extra

    set_grad_sink(False)
    cls = getattr(importlib.import_module(f"autoformer_amd.factory.{name}"), name)
    m = cls(44, 256, 512, freq)
    det_init_(m)
    m = m.to(DEV).train()
    Dm = None
    if disc:
        from autoformer_amd.factory.Discriminator import Discriminator
        Dm = Discriminator(crop_len=T)
        det_init_(Dm)
        Dm = Dm.to(DEV).train()
    x, e = _synthetic(B, T)
    mods = [m] + ([Dm] if disc else [])
    bufs = [{k: v.clone() for k, v in mod.state_dict().items()} for mod in mods]

    def restore():  # parameters and BN running stats back to the same start
        for mod, b in zip(mods, bufs):
            mod.load_state_dict(b)

    A.set_compute("fp32")
    l32, p32, g32 = _fwd_bwd(m, x, e, Dm)
    # intrinsic sensitivity: the same fp32 step on weights rounded to bf16 (what bf16 compute
    # starts from).  A gradient that moves this much under weight rounding alone cannot be
    # held tighter than that in bf16.
    with torch.no_grad():
        for mod in mods:
            for q in mod.parameters():
                q.copy_(q.bfloat16().float())
    _, _, g32r = _fwd_bwd(m, x, e, Dm)
    restore()
    A.set_compute("bf16")
    l16, p16, g16 = _fwd_bwd(m, x, e, Dm)
    r = rel_inf(p16.cpu(), p32.cpu())
    assert np.isfinite(l16) and abs(l16 - l32) <= 5e-2 * abs(l32), (l16, l32)
    assert r <= 5e-2, r
    devs, sens = {}, {}
    for n, g in g32.items():
        h = g16[n]
        assert torch.isfinite(h).all(), n
        if _bn_fed_bias(n):
            continue
        nrm = g.norm().clamp_min(1e-12)
        devs[n] = ((h - g).norm() / nrm).item()
        sens[n] = ((g32r[n] - g).norm() / nrm).item()
    top = sorted(devs.items(), key=lambda kv: -kv[1])
    print(f"\n{name}{'+D' if disc else ''} B={B} T={T}: loss fp32 {l32:.5f} bf16 {l16:.5f}, mel_postnet rel-inf "
          f"{r:.2e}; grad rel-Frobenius bf16 vs fp32: median {np.median(list(devs.values())):.3e}; fp32 on "
          f"bf16-rounded weights vs fp32: median {np.median(list(sens.values())):.3e}; top (bf16 / rounded): "
          + ", ".join(f"{n} {v:.3f}/{sens[n]:.3f}" for n, v in top[:10]))
    bad = {n: (v, sens[n]) for n, v in devs.items() if v > max(GRAD_BAR, SENS_FACTOR * sens[n])}
    assert not bad, bad
    ts = TrainStep(m, lr=1e-4, extra=gan_extra(Dm) if disc else None, extra_modules=[Dm] if disc else ())
    try:
        losses = [float(ts.step(x, e).item()) for _ in range(3)]
        ts.check()
    finally:
        set_grad_sink(False)
    assert all(np.isfinite(losses)) and losses[2] < losses[0], losses


@pytest.mark.timeout(300)
def test_c2_autovc_b64_t128_bf16_vs_fp32():
    _check("AutoVC", 16, 64, 128)


@pytest.mark.timeout(300)
def test_c4_metaconv_b64_t176_bf16_vs_fp32():
    _check("MetaConv", 22, 64, 176)


@pytest.mark.timeout(300)
def test_c5_autovc_disc_b64_t176_bf16_vs_fp32():
    _check("AutoVC", 22, 64, 176, disc=True)
