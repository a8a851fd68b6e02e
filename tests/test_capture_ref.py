"""CPU checks of the fp64 restatements used by the full-size op capture (tests/capture_ref.py):
the avc_operand window materialisation against F.conv1d, and the LSTM forward / backward
references against torch.nn.LSTM and its autograd."""
import torch

from autoformer_amd import _lib as L
from tests.capture_ref import lstm_bwd_ref, lstm_fwd_ref, materialize


def _op(t, ld, kstrided=0, window=None):
    o = L.Operand()
    o._keep = t
    o.ptr = t.data_ptr()
    o.dtype = L.F32
    o.kstrided = kstrided
    o.ld = ld
    o.batch_stride = 0
    if window:
        o.taps, o.pad, o.t_out, o.t_in, o.chans = window
    return o


def test_window_is_conv1d():
    torch.manual_seed(0)
    B, T, Ci, Co, k = 3, 11, 6, 5, 5
    x = torch.randn(B, Ci, T, dtype=torch.float64)
    w = torch.randn(Co, Ci, k, dtype=torch.float64)
    ref = torch.nn.functional.conv1d(x, w, padding=2)  # (B, Co, T)
    xf = x.transpose(1, 2).reshape(B * T, Ci).float().contiguous()
    A = materialize(_op(xf, Ci, window=(k, 2, T, T, Ci)), B * T, k * Ci)
    Wp = w.permute(0, 2, 1).reshape(Co, k * Ci)  # [co][tap*Ci + ci]
    got = (A @ Wp.t()).view(B, T, Co).transpose(1, 2)
    assert (got - ref).abs().max() < 1e-4
    # the same window as a K-strided operand (frames along K): its transpose
    At = materialize(_op(xf, Ci, kstrided=1, window=(k, 2, T, T, Ci)), k * Ci, B * T)
    assert torch.equal(At, A.t())
    # plain row-major / K-strided views
    m = torch.randn(4, 7)
    assert torch.equal(materialize(_op(m, 7), 4, 7), m.double())
    assert torch.equal(materialize(_op(m, 7, kstrided=1), 7, 4), m.double().t())


def test_lstm_refs_match_torch():
    torch.manual_seed(1)
    B, T, In, H = 2, 7, 5, 4
    lstm = torch.nn.LSTM(In, H, batch_first=True, bidirectional=True).double()
    x = torch.randn(B, T, In, dtype=torch.float64, requires_grad=True)
    out, _ = lstm(x)
    ws = [(lstm.weight_ih_l0, lstm.bias_ih_l0 + lstm.bias_hh_l0, lstm.weight_hh_l0),
          (lstm.weight_ih_l0_reverse, lstm.bias_ih_l0_reverse + lstm.bias_hh_l0_reverse, lstm.weight_hh_l0_reverse)]
    xp = torch.cat([x.reshape(B * T, In) @ wi.t() + b for wi, b, _ in ws], 1).detach()
    whh = torch.cat([wh for _, _, wh in ws], 0).detach()
    h, c, g = lstm_fwd_ref(xp, whh, B, T, H, 2)
    assert (h.view(B, T, 2 * H) - out.detach()).abs().max() < 1e-12
    dout = torch.randn_like(out)
    out.backward(dout)
    dG = lstm_bwd_ref(dout.reshape(B * T, 2 * H), c, g, whh, B, T, H, 2)
    xs = x.detach().reshape(B * T, In)
    for d, wi in enumerate((lstm.weight_ih_l0, lstm.weight_ih_l0_reverse)):
        dW = dG[:, d * 4 * H:(d + 1) * 4 * H].t() @ xs
        assert (dW - wi.grad).abs().max() < 1e-10
