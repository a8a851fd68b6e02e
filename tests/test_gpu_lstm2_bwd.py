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
