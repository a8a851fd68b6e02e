"""Host logic of the fused loss block (train._VCLossFn, train.py:84-96 of the reference): which
upstream gradients reach avc_vc_loss_grad and which input gradients come back.  The two
kernels are replaced by torch restatements of their documented contracts
(include/autovc_hip.h: avc_vc_loss / avc_vc_loss_grad), so this runs on the CPU; the kernels
themselves are checked on the GPU (tests/test_gpu_kernels.py::test_vc_loss_block_matches_torch)."""
import pytest
import torch
import torch.nn.functional as F


def _fake_vc_loss(x, y1, y2, ca, cb, lam):
    m0 = ((x - y1) ** 2).mean()
    m1 = ((x - y2) ** 2).mean()
    m2 = (ca - cb).abs().mean() if ca.numel() else torch.zeros(())
    return torch.stack([m0, m1, m2, m0 + m1 + lam * m2])


def _fake_vc_loss_grad(x, y1, y2, ca, cb, lam, d, need):
    def val(t):
        return t if t is not None else torch.zeros(())
    d0, d1, d2, d3 = (val(t) for t in d)
    n1, n2 = x.numel(), max(ca.numel(), 1)
    g1 = (d3 + d0) * 2 * (y1 - x) / n1
    g2 = (d3 + d1) * 2 * (y2 - x) / n1
    ga = (lam * d3 + d2) * torch.sign(ca - cb) / n2
    outs = (g1, g2, ga, -ga)
    return [o if nd else None for o, nd in zip(outs, need)]


@pytest.fixture
def fused(monkeypatch):
    from autoformer_amd import kernels as K
    from autoformer_amd import train

    monkeypatch.setattr(K, "vc_loss", _fake_vc_loss)
    monkeypatch.setattr(K, "vc_loss_grad", _fake_vc_loss_grad)
    return train.vc_loss_block


@pytest.mark.parametrize("combo", ["total", "total+parts", "parts_only"])
def test_loss_block_gradient_routing(fused, combo):
    torch.manual_seed(0)
    x = torch.randn(2, 16, 80)
    y1 = torch.randn(2, 1, 16, 80, requires_grad=True)
    y2 = torch.randn(2, 1, 16, 80, requires_grad=True)
    ca = torch.randn(2, 88, requires_grad=True)
    cb = torch.randn(2, 88, requires_grad=True)
    lam = 0.6
    total, (l_id, l_ps, l_cd) = fused(x, y1.squeeze(), y2.squeeze(), ca, cb, lam)
    y1r, y2r, car, cbr = (t.detach().clone().requires_grad_(True) for t in (y1, y2, ca, cb))
    r_id = F.mse_loss(x, y1r.squeeze())
    r_ps = F.mse_loss(x, y2r.squeeze())
    r_cd = F.l1_loss(car, cbr)
    r_tot = r_id + r_ps + lam * r_cd
    for a, b in ((total, r_tot), (l_id, r_id), (l_ps, r_ps), (l_cd, r_cd)):
        torch.testing.assert_close(a, b)
    if combo == "total":
        total.backward()
        r_tot.backward()
    elif combo == "total+parts":
        (1.5 * total + 0.25 * l_id + 2.0 * l_cd).backward()
        (1.5 * r_tot + 0.25 * r_id + 2.0 * r_cd).backward()
    else:
        (l_ps + 3.0 * l_cd).backward()
        (r_ps + 3.0 * r_cd).backward()
    for a, b in ((y1, y1r), (y2, y2r), (ca, car), (cb, cbr)):
        torch.testing.assert_close(a.grad, b.grad)


def test_loss_block_x_real_gradient(fused):
    """x_real is data in train.py, but a caller that makes it a leaf still gets -(g1 + g2)."""
    torch.manual_seed(1)
    x = torch.randn(3, 8, 80, requires_grad=True)
    y1, y2 = torch.randn(3, 8, 80), torch.randn(3, 8, 80)
    ca, cb = torch.randn(3, 44), torch.randn(3, 44)
    total, _ = fused(x, y1, y2, ca, cb, 1.0)
    total.backward()
    xr = x.detach().clone().requires_grad_(True)
    (F.mse_loss(xr, y1) + F.mse_loss(xr, y2) + F.l1_loss(ca, cb)).backward()
    torch.testing.assert_close(x.grad, xr.grad)
