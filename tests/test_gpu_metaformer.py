"""MetaConv / MetaPool on the MI355X.

Kernel numerics: each new HIP kernel (GroupNorm(1), LayerNorm, GELU backward, pooling
token mixer, patchify, batched transpose, the fused MLP-Mixer) against a plain PyTorch fp32
computation of the same op.  Model parity: one train.py step (forward, encoder re-pass, 2xMSE
+ L1, backward) against the reference goldens tests/golden/meta{conv,pool}_T176.npz.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from .helpers import bn_state_mismatches, grad_mismatches, rel_inf, to_dev

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(autouse=True)
def _fp32():
    import autoformer_amd as A

    A.set_compute("fp32")
    yield


def _t(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(DEV)


def _frames_to_bcl(x, B, L):
    return x.view(B, L, -1).transpose(1, 2)


# ------------------------------------------------------------------------------------ kernels
@pytest.mark.parametrize("B,L,C", [(2, 176, 512), (3, 344, 344), (1, 7, 5)])
def test_group_norm_fwd_bwd(B, L, C):
    from autoformer_amd import metaformer as MF

    gn = torch.nn.GroupNorm(1, C).to(DEV)
    with torch.no_grad():
        gn.weight.copy_(_t(C, seed=1) * 0.5 + 1)
        gn.bias.copy_(_t(C, seed=2) * 0.1)
    x = _t(B * L, C, seed=3, scale=2.0).add_(0.7).requires_grad_()
    dy = _t(B * L, C, seed=4)
    y = MF.group_norm(x, B, gn)
    y.backward(dy)
    xr = x.detach().clone().requires_grad_()
    gw, gb = gn.weight.grad.clone(), gn.bias.grad.clone()
    gn.zero_grad()
    yr = gn(_frames_to_bcl(xr, B, L)).transpose(1, 2).reshape(B * L, C)
    yr.backward(dy)
    torch.testing.assert_close(y, yr, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(x.grad, xr.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(gw, gn.weight.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(gb, gn.bias.grad, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("R,D", [(242, 176), (3698, 344), (5, 3)])
def test_layer_norm_fwd_bwd(R, D):
    from autoformer_amd import kernels as K

    w, b = _t(D, seed=1) * 0.3 + 1, _t(D, seed=2) * 0.1
    x = _t(R, D, seed=3, scale=3.0)
    dy = _t(R, D, seed=4)
    y, mean, rstd = K.layer_norm_fwd(x, w, b, 1e-5)
    dg, db = torch.empty(D, device=DEV), torch.empty(D, device=DEV)
    dx = K.layer_norm_bwd(dy, x, w, mean, rstd, dg, db)
    xr, wr, br = (t.clone().requires_grad_() for t in (x, w, b))
    yr = F.layer_norm(xr, (D,), wr, br, 1e-5)
    yr.backward(dy)
    torch.testing.assert_close(y, yr, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(dx, xr.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(dg, wr.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(db, br.grad, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("R,D", [(242, 176), (3698, 344), (130, 512), (67, 12)])
def test_layer_norm_bf16_and_residual_forms(R, D):
    """avc_layer_norm_fwd2 with a bf16-only output and avc_layer_norm_bwd2 with the residual branch's
    gradient added and the bf16 twin written (the mixer's LN -> add chains, MLPMixer.py:80-86),
    dx and the parameter sums from the one-pass kernel, accumulate on."""
    import autoformer_amd as A
    from autoformer_amd import kernels as K

    prev = "bf16" if K.compute() == K.BF16 else "fp32"
    A.set_compute("bf16")  # the bf16 twins exist in bf16 compute mode only
    try:
        _ln_forms(K, R, D)
    finally:
        A.set_compute(prev)


def _ln_forms(K, R, D):
    w, b = _t(D, seed=1) * 0.3 + 1, _t(D, seed=2) * 0.1
    x = _t(R, D, seed=3, scale=3.0)
    dy, res = _t(R, D, seed=4), _t(R, D, seed=5)
    y16, mean, rstd = K.layer_norm_fwd(x, w, b, 1e-5, out_bf16=True)
    assert y16.dtype == torch.bfloat16
    dg, db = _t(D, seed=6), _t(D, seed=7)
    dg0, db0 = dg.clone(), db.clone()
    rsum = torch.empty(R, device=DEV)
    dx = K.layer_norm_bwd(dy, x, w, mean, rstd, dg, db, accumulate=True, residual=res, twin=True, row_sum=rsum)
    xr, wr, br = (t.clone().requires_grad_() for t in (x, w, b))
    yr = F.layer_norm(xr, (D,), wr, br, 1e-5)
    yr.backward(dy)
    torch.testing.assert_close(y16.float(), yr, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(dx, xr.grad + res, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(dx._bf16.float(), xr.grad + res, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(rsum, (xr.grad + res).sum(1), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dg, dg0 + wr.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(db, db0 + br.grad, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("B,L,C", [(2, 176, 512), (3, 344, 344)])
def test_group_norm_twin(B, L, C):
    import autoformer_amd as A
    from autoformer_amd import kernels as K

    x = _t(B * L, C, seed=3, scale=2.0)
    w, b = _t(C, seed=1) * 0.5 + 1, _t(C, seed=2) * 0.1
    prev = "bf16" if K.compute() == K.BF16 else "fp32"
    A.set_compute("bf16")
    try:
        y, _, _ = K.group_norm_fwd(x, B, C, w, b, 1e-5, twin=True)
    finally:
        A.set_compute(prev)
    yr = F.group_norm(_frames_to_bcl(x, B, L), 1, w, b, 1e-5).transpose(1, 2).reshape(B * L, C)
    torch.testing.assert_close(y, yr, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(y._bf16.float(), yr, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("B,R,C,ld", [(2, 1849, 344, 1856), (3, 121, 176, 128), (1, 7, 5, 8)])
def test_transpose_pad_bf16_source(B, R, C, ld):
    """avc_transpose_batched2 from a bf16 source (the LayerNorm's bf16 output) into padded rows."""
    from autoformer_amd import kernels as K

    x = _t(B * R, C, seed=12).bfloat16()
    y = K.transpose_pad(x, B, R, C, ld, dtype=K.BF16)
    ref = torch.zeros(B, C, ld, device=DEV, dtype=torch.bfloat16)
    ref[:, :, :R] = x.view(B, R, C).transpose(1, 2)
    torch.testing.assert_close(y.view(B, C, ld), ref, rtol=0, atol=0)


def test_gelu_fwd_bwd():
    from autoformer_amd import kernels as K

    x = _t(1000, 37, seed=5, scale=3.0)
    g = _t(1000, 37, seed=6)
    xr = x.clone().requires_grad_()
    yr = F.gelu(xr)
    yr.backward(g)
    torch.testing.assert_close(K.act_fwd(x, K.ACT_GELU), yr, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(K.gelu_bwd(g, x), xr.grad, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("B,L,C", [(2, 176, 512), (1, 2, 3), (2, 1, 4)])
def test_pool_mixer_fwd_bwd(B, L, C):
    from autoformer_amd import metaformer as MF

    x = _t(B * L, C, seed=7).requires_grad_()
    dy = _t(B * L, C, seed=8)
    y = MF.pool_mixer(x, B, L)
    y.backward(dy)
    # reference on the CPU in fp64 (contiguous (B, C, L) input)
    xr = x.detach().cpu().double().requires_grad_()
    xb = xr.view(B, L, C).transpose(1, 2).contiguous()
    yr = (F.avg_pool1d(xb, 3, 1, 1, count_include_pad=False) - xb).transpose(1, 2).reshape(B * L, C)
    yr.backward(dy.cpu().double())
    torch.testing.assert_close(y.cpu().double(), yr, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(x.grad.cpu().double(), xr.grad, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("B,L,C,ps", [(2, 176, 176, 16), (2, 344, 344, 8), (1, 16, 8, 4)])
def test_patchify_roundtrip(B, L, C, ps):
    from autoformer_amd import kernels as K

    x = _t(B * L, C, seed=9)
    P = K.patchify(x, B, L, C, ps)
    img = _frames_to_bcl(x, B, L)  # (B, C=H, L=W)
    ref = img.reshape(B, C // ps, ps, L // ps, ps).permute(0, 1, 3, 2, 4).reshape(B * (C // ps) * (L // ps), ps * ps)
    torch.testing.assert_close(P, ref, rtol=0, atol=0)
    back = K.patchify(P, B, L, C, ps, backward=True)
    torch.testing.assert_close(back, x, rtol=0, atol=0)
    P16 = K.patchify(x, B, L, C, ps, out_bf16=True)  # the bf16 form: the rounding of the same rearrangement
    assert P16.dtype == torch.bfloat16
    torch.testing.assert_close(P16, ref.to(torch.bfloat16), rtol=0, atol=0)


@pytest.mark.parametrize("B,R,C", [(2, 176, 344), (3, 7, 5), (1, 344, 88)])
def test_transpose_batched(B, R, C):
    from autoformer_amd import kernels as K

    x = _t(B * R, C, seed=10)
    y = K.transpose_batched(x, B, R, C).view(B, C, R)
    torch.testing.assert_close(y, x.view(B, R, C).transpose(1, 2), rtol=0, atol=0)
    acc = _t(B * C * R, seed=11)
    y2 = K.transpose_batched(x, B, R, C, out=acc.clone(), accumulate=True)
    torch.testing.assert_close(y2, acc + x.view(B, R, C).transpose(1, 2).reshape(-1), rtol=1e-6, atol=1e-6)


def _torch_mixer(mix, img):
    """Plain PyTorch fp32 MLP-Mixer (MLPMixer.py:58-92, depth 1) on img (B, 1, H, W)."""
    ps = mix.ps
    B, _, H, W = img.shape
    p = img.reshape(B, H // ps, ps, W // ps, ps).permute(0, 1, 3, 2, 4).reshape(B, (H // ps) * (W // ps), ps * ps)
    z = F.linear(p, mix[1].weight, mix[1].bias)
    tok, ch = mix[2][0], mix[2][1]
    y = F.layer_norm(z, z.shape[-1:], tok.norm.weight, tok.norm.bias, tok.norm.eps)
    y = F.conv1d(F.gelu(F.conv1d(y, tok.fn[0].weight, tok.fn[0].bias)), tok.fn[3].weight, tok.fn[3].bias)
    z = z + y
    y = F.layer_norm(z, z.shape[-1:], ch.norm.weight, ch.norm.bias, ch.norm.eps)
    z = z + F.linear(F.gelu(F.linear(y, ch.fn[0].weight, ch.fn[0].bias)), ch.fn[3].weight, ch.fn[3].bias)
    return F.conv1d(z, mix[3].weight, mix[3].bias, padding=mix[3].padding)


@pytest.mark.parametrize("B,L,ps,out", [(2, 176, 16, 88), (2, 344, 8, 88)])
def test_mlp_mixer_vs_torch(B, L, ps, out):
    from autoformer_amd import metaformer as MF
    from autoformer_amd.factory.MLPMixer import MLPMixer

    torch.manual_seed(0)
    mix = MLPMixer(image_size=L, channels=1, patch_size=ps, dim=L, depth=1, out_dim=out).to(DEV)
    x = _t(B * L, L, seed=12).requires_grad_()
    dy = _t(B * L, out, seed=13)
    y = MF.mlp_mixer(x, mix, B, L)
    y.backward(dy)
    grads = {n: p.grad.clone() for n, p in mix.named_parameters()}
    mix.zero_grad()
    xr = x.detach().clone().requires_grad_()
    yr = _torch_mixer(mix, _frames_to_bcl(xr, B, L).unsqueeze(1))  # (B, out, L)
    yr.transpose(1, 2).reshape(B * L, out).backward(dy)
    assert rel_inf(y.detach().cpu(), yr.transpose(1, 2).reshape(B * L, out).detach().cpu()) < 1e-4
    assert rel_inf(x.grad.cpu(), xr.grad.cpu()) < 1e-4
    for n, p in mix.named_parameters():
        assert rel_inf(grads[n].cpu(), p.grad.cpu()) < 1e-4, n


@pytest.mark.parametrize("comp,dim", [("fp32", 90), ("fp32", 516), ("bf16", 90), ("bf16", 516), ("bf16", 768)])
def test_mlp_mixer_general_dim(comp, dim):
    """A mixer dim outside the one-pass LayerNorm forms (D % 4 != 0, or D > 512: the reference
    MetaDV's dim=768) takes the plain LayerNorm + add / convert passes, in both compute
    modes, against plain PyTorch fp32."""
    import autoformer_amd as A
    from autoformer_amd import metaformer as MF
    from autoformer_amd.factory.MLPMixer import MLPMixer

    A.set_compute(comp)
    torch.manual_seed(0)
    B, L, ps, out = 2, 176, 16, 88
    mix = MLPMixer(image_size=L, channels=1, patch_size=ps, dim=dim, depth=1, out_dim=out).to(DEV)
    x = _t(B * L, L, seed=12).requires_grad_()
    dy = _t(B * dim, out, seed=13)
    y = MF.mlp_mixer(x, mix, B, L)
    y.backward(dy)
    torch.cuda.synchronize()
    grads = {n: p.grad.clone() for n, p in mix.named_parameters()}
    mix.zero_grad()
    xr = x.detach().clone().requires_grad_()
    yr = _torch_mixer(mix, _frames_to_bcl(xr, B, L).unsqueeze(1))  # (B, out, dim)
    yr.transpose(1, 2).reshape(B * dim, out).backward(dy)
    yr2 = yr.transpose(1, 2).reshape(B * dim, out).detach()
    if comp == "fp32":
        assert rel_inf(y.detach().cpu(), yr2.cpu()) < 1e-4
        assert rel_inf(x.grad.cpu(), xr.grad.cpu()) < 1e-4
        for n, p in mix.named_parameters():
            assert rel_inf(grads[n].cpu(), p.grad.cpu()) < 1e-4, n
    else:  # bf16 operands: relative Frobenius at bf16 rounding scale
        def rel(a, b):
            return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()

        assert rel(y.detach(), yr2) < 2e-2
        assert rel(x.grad, xr.grad) < 3e-2
        for n, p in mix.named_parameters():
            assert rel(grads[n], p.grad) < 5e-2, n


# ------------------------------------------------------------------------------------ models
def _model(kind, comp="fp32"):
    import autoformer_amd as A
    from autoformer_amd.detinit import det_init_

    A.set_compute(comp)
    if kind == "metaconv":
        from factory.MetaConv import MetaConv as M
    else:
        from factory.MetaPool import MetaPool as M
    m = M(44, 256, 512, 22)
    det_init_(m)
    return m.to(DEV).train()


def _step(m, x, e):
    x_id, x_psnt, code = m(x, e, e)
    l1 = F.mse_loss(x, x_id.squeeze())
    l2 = F.mse_loss(x, x_psnt.squeeze())
    code_re = m(x_psnt, e, None)
    l3 = F.l1_loss(code, code_re)
    return (x_id, x_psnt, code, code_re), (l1, l2, l3), l1 + l2 + l3


@pytest.mark.parametrize("kind", ["metaconv", "metapool"])
def test_metaformer_fp32_matches_reference_goldens(golden, kind):
    g = golden(f"{kind}_T176.npz")
    m = _model(kind)
    x, e = to_dev(g, DEV, "x", "emb")
    outs, losses, total = _step(m, x, e)
    m.zero_grad()
    total.backward()
    torch.cuda.synchronize()
    for o, k in zip(outs, ("mel", "mel_psnt", "codes", "codes_re")):
        assert rel_inf(o.detach().cpu(), g[k]) < 1e-3, k
    np.testing.assert_allclose([l.item() for l in losses], g["losses"], rtol=1e-4)
    # The reference's own fp32 gradients sit up to 1.4e-2 (head, relative to max|head|) and
    # 4e-4 (norm) away from an fp64 evaluation of the same step (measured with the oracle in
    # fp64), so heads are held to 5e-2 and norms to 1e-2.  Analytically-zero gradients: conv
    # biases feeding a training-mode BN (incl. postnet.convolutions.4), and for MetaPool the
    # GroupNorm bias norm1.bias (a per-channel constant is annihilated by pool(x) - x).
    def zero_grad(n):
        return "conv.bias" in n or (kind == "metapool" and n.endswith("norm1.bias"))

    # MetaPool's heads are chaotic at B=2: 1 ulp of noise on the norm outputs of the fp32 oracle
    # itself moves them by up to 2.8 % of the tensor scale (ReLU decisions near 0 flip; MetaConv:
    # 0.6 %; profiles/r4_metaformer_flip_spread.txt).  The GPU's worst head sits at 2.9 % (round 5,
    # profiles/r5_metapool_heads.txt; decoder.output_conv_2.1.bias, 6 % in round 4, at 0.8 %): both
    # families are held to the 5e-2 head bar, norms to 1e-2
    bad = grad_mismatches(m, g, tol=1e-2, head_tol=5e-2, bn_fed_bias=zero_grad)
    assert not bad, sorted(bad.items())
    assert not bn_state_mismatches(m, g)


@pytest.mark.parametrize("kind", ["metaconv", "metapool"])
def test_metaformer_bf16_loose(golden, kind):
    g = golden(f"{kind}_T176.npz")
    m = _model(kind, "bf16")
    x, e = to_dev(g, DEV, "x", "emb")
    outs, losses, total = _step(m, x, e)
    total.backward()
    torch.cuda.synchronize()
    assert rel_inf(outs[1].detach().cpu(), g["mel_psnt"]) < 5e-2
    np.testing.assert_allclose([l.item() for l in losses], g["losses"], rtol=5e-2)
    for p in m.parameters():
        assert torch.isfinite(p.grad).all()


def test_metaconv_rejects_wrong_crop():
    m = _model("metaconv")
    x = torch.zeros(2, 128, 80, device=DEV)
    e = torch.zeros(2, 256, device=DEV)
    with pytest.raises((RuntimeError, IndexError)):
        m(x, e, e)
