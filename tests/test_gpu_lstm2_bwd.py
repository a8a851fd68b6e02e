"""The decoder lstm2 backward as ONE two-layer wavefront launch (avc_lstm2_bwd, lstm.hip
lstm2_persist_bwd; AutoVC.py:96,110's nn.LSTM(512, 1024, 2)) against the same backward as two
single-layer persistent launches with the dX1 = dG1 W_ih1 GEMM between them (the path it replaces),
and the whole step's gradients with the wavefront on / off.  Both use bf16 payloads and weights with
fp32 accumulation; they differ only in the order of the fp32 sums."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("B,T", [(64, 128), (48, 40)])
def test_lstm2_wavefront_backward_matches_two_launches(B, T):
    import autoformer_amd as A
    from autoformer_amd import kernels as K
    from autoformer_amd import layers as Ly

    A.set_compute("bf16")
    if not K.lstm2_bwd_persistent(B, 1024):
        pytest.skip("the wavefront backward grid is not resident on this device")
    torch.manual_seed(B + T)
    mod = torch.nn.LSTM(512, 1024, 2, batch_first=True).to(DEV)
    cores = [Ly.LSTMLayerCore(mod, layer) for layer in range(2)]
    x = (torch.randn(B * T, 512, device=DEV) * 0.5).requires_grad_(True)
    gy = torch.randn(B * T, 1024, device=DEV) * 0.1
    res = []
    saved = Ly._PAIR_BWD
    try:
        for on in (True, False):
            Ly._PAIR_BWD = on
            mod.zero_grad(set_to_none=True)
            x.grad = None
            Ly.set_grad_sink(False)
            y = Ly.lstm(mod, cores, x, B, T)
            (y.float() * gy).sum().backward()
            torch.cuda.synchronize()
            res.append((x.grad.clone(), [p.grad.clone() for p in mod.parameters()]))
        K.check_faults()
    finally:
        Ly._PAIR_BWD = saved
    (dxa, ga), (dxb, gb) = res
    assert _rel(dxa, dxb) < 2e-3, _rel(dxa, dxb)
    for (n, _), p, q in zip(mod.named_parameters(), ga, gb):
        assert _rel(p, q) < 2e-3, (n, _rel(p, q))


def test_lstm2_wavefront_bias_partials_and_bf16_only_outputs():
    """ABI 28: the bf16-only form writes the same bf16 dG as the fp32 + twin form, and its per-group
    partials (dG summed over each 16-utterance group and every step) match the fp32 dG's sums."""
    import autoformer_amd as A
    from autoformer_amd import kernels as K

    A.set_compute("bf16")
    B, T, H = 48, 24, 1024
    if not K.lstm2_bwd_persistent(B, H):
        pytest.skip("the wavefront backward grid is not resident on this device")
    g = torch.Generator(device=DEV).manual_seed(5)
    dh = torch.randn(B * T, H, device=DEV, generator=g) * 0.1
    cs = [torch.randn(B * T, H, device=DEV, generator=g) * 0.5 for _ in range(2)]
    gs = [torch.rand(B * T, 4 * H, device=DEV, generator=g) for _ in range(2)]
    ws = [(torch.randn(H, 4 * H, device=DEV, generator=g) * 0.02).bfloat16() for _ in range(3)]
    d0, d1 = K.lstm2_bwd(dh, cs[0], gs[0], cs[1], gs[1], *ws, B, T, H)
    e0, e1, dbp = K.lstm2_bwd(dh, cs[0], gs[0], cs[1], gs[1], *ws, B, T, H, fp32=False, db=True)
    torch.cuda.synchronize()
    K.check_faults()
    assert e0.dtype == torch.bfloat16 and torch.equal(e0, d0._bf16) and torch.equal(e1, d1._bf16)
    ng = -(-B // 16)
    for layer, d in ((0, d0), (1, d1)):
        ref = torch.zeros(ng * 16, T, 4 * H, device=DEV, dtype=torch.float64)
        ref[:B] = d.double().view(B, T, 4 * H)
        assert _rel(dbp[layer], ref.view(ng, 16 * T, 4 * H).sum(1)) < 1e-5
