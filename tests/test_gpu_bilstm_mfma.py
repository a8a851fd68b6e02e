"""The encoder BiLSTM on MFMA (lstm_mfma_fwd / lstm_mfma_bwd, csrc/lstm.hip; reference
factory/AutoVC.py:43,54-55 -- nn.LSTM(512, 44, 2, batch_first=True, bidirectional=True)) against a
float64 PyTorch restatement of the recurrence on the same inputs.

bf16 compute: W_hh and the recurrent h / dG operands are bf16, the gates, cell state and the
accumulation fp32, so the bar is the bf16 one of the other recurrences (rel-Frobenius <= 1e-2 per
output at the bench shape B=64, T=128; the capture tests hold the decoder LSTMs to the same bar).
Ragged batches (B not a multiple of the 4 utterances of a workgroup) and every instantiated H
are covered."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def relf(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return float((a - b).norm() / max(b.norm().item(), 1e-30))


def ref_fwd(xp, w, B, T, H, dirs):
    """xp (B, T, dirs*4H), w (dirs*4H, H): h, c, activated gates, all (B, T, dirs*.) float64."""
    G = 4 * H
    h = torch.zeros(B, T, dirs * H, dtype=torch.float64)
    c = torch.zeros_like(h)
    g = torch.zeros(B, T, dirs * G, dtype=torch.float64)
    for d in range(dirs):
        W = w[d * G:(d + 1) * G]
        hp = torch.zeros(B, H, dtype=torch.float64)
        cp = torch.zeros_like(hp)
        for s in range(T):
            t = T - 1 - s if d else s
            pre = xp[:, t, d * G:(d + 1) * G] + hp @ W.t()
            i, f, gg, o = torch.sigmoid(pre[:, :H]), torch.sigmoid(pre[:, H:2 * H]), torch.tanh(
                pre[:, 2 * H:3 * H]), torch.sigmoid(pre[:, 3 * H:])
            cp = f * cp + i * gg
            hp = o * torch.tanh(cp)
            h[:, t, d * H:(d + 1) * H] = hp
            c[:, t, d * H:(d + 1) * H] = cp
            g[:, t, d * G:(d + 1) * G] = torch.cat([i, f, gg, o], 1)
    return h, c, g


def ref_bwd(dh_out, c, g, w, B, T, H, dirs):
    """dL/d(pre-activation gates) (B, T, dirs*4H) float64 from the forward's c and activated gates."""
    G = 4 * H
    dg = torch.zeros(B, T, dirs * G, dtype=torch.float64)
    for d in range(dirs):
        W = w[d * G:(d + 1) * G]
        dgn = torch.zeros(B, G, dtype=torch.float64)
        dc = torch.zeros(B, H, dtype=torch.float64)
        for s in range(T):
            t = s if d else T - 1 - s  # opposite to the forward
            tp = t + 1 if d else t - 1
            gt = g[:, t, d * G:(d + 1) * G]
            i, f, gg, o = gt[:, :H], gt[:, H:2 * H], gt[:, 2 * H:3 * H], gt[:, 3 * H:]
            ct = c[:, t, d * H:(d + 1) * H]
            cp = c[:, tp, d * H:(d + 1) * H] if 0 <= tp < T else torch.zeros_like(ct)
            dh = dh_out[:, t, d * H:(d + 1) * H] + dgn @ W
            tc = torch.tanh(ct)
            dcs = dc + dh * o * (1 - tc * tc)
            dgn = torch.cat([dcs * gg * i * (1 - i), dcs * cp * f * (1 - f), dcs * i * (1 - gg * gg),
                             dh * tc * o * (1 - o)], 1)
            dc = dcs * f
            dg[:, t, d * G:(d + 1) * G] = dgn
    return dg


@pytest.mark.parametrize("B,T,H,dirs", [(64, 128, 44, 2), (3, 33, 44, 2), (7, 20, 44, 1), (5, 17, 16, 1),
                                        (6, 21, 64, 2), (4, 9, 32, 2), (2, 11, 48, 1)])
def test_bilstm_mfma_matches_fp64(B, T, H, dirs):
    import autoformer_amd as A
    from autoformer_amd import _lib as L
    from autoformer_amd import kernels as K

    A.set_compute("bf16")
    L.lib().avc_lstm_set_small_mfma(1)
    try:
        assert L.lib().avc_lstm_small_mfma(H, K.BF16) == 1
        g0 = torch.Generator().manual_seed(B * 1000 + T + H)
        G = 4 * H
        xp = torch.randn(B, T, dirs * G, generator=g0) * 0.8
        w = (torch.rand(dirs * G, H, generator=g0) * 2 - 1) / H ** 0.5
        h, c, g = K.lstm_fwd(xp.reshape(B * T, -1).to(DEV), w.to(DEV), B, T, H, dirs)
        torch.cuda.synchronize()
        hr, cr, gr = ref_fwd(xp.double(), w.double(), B, T, H, dirs)
        res = {"h": relf(h, hr.reshape(B * T, -1)), "c": relf(c, cr.reshape(B * T, -1)),
               "gates": relf(g, gr.reshape(B * T, -1))}
        assert torch.equal(h._bf16, h.bfloat16()), "bf16 twin of h"
        dh = torch.randn(B, T, dirs * H, generator=g0)
        dg = K.lstm_bwd(dh.reshape(B * T, -1).to(DEV), h, c, g, w.to(DEV), None, B, T, H, dirs)
        torch.cuda.synchronize()
        # the reference backward runs from the GPU forward's own c / gates (isolates the backward)
        dgr = ref_bwd(dh.double(), c.cpu().double().reshape(B, T, -1), g.cpu().double().reshape(B, T, -1),
                      w.double(), B, T, H, dirs)
        res["dG"] = relf(dg, dgr.reshape(B * T, -1))
        assert torch.equal(dg._bf16, dg.bfloat16()), "bf16 twin of dG"
        bad = {k: v for k, v in res.items() if not v < 1e-2}
        assert not bad, (res, bad)
    finally:
        L.lib().avc_lstm_set_small_mfma(-1)
        A.set_compute("fp32")


def test_bilstm_mfma_selection():
    """Off by default (measured slower, profiles/r6_bilstm_mfma_ab.txt); selectable in bf16 mode only."""
    import os

    from autoformer_amd import _lib as L
    from autoformer_amd import kernels as K

    if not os.environ.get("AVC_BILSTM_MFMA"):
        assert L.lib().avc_lstm_small_mfma(44, K.BF16) == 0
    L.lib().avc_lstm_set_small_mfma(1)
    try:
        assert L.lib().avc_lstm_small_mfma(44, K.F32) == 0  # fp32 parity mode keeps the FMA kernels
        assert L.lib().avc_lstm_small_mfma(44, K.BF16) == 1
        assert L.lib().avc_lstm_small_mfma(40, K.BF16) == 0  # not instantiated: packed-FMA kernels
    finally:
        L.lib().avc_lstm_set_small_mfma(-1)
