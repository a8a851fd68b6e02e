"""The decoder lstm1 with its input projection folded per code and per utterance
(layers._LSTM1FoldFn) against the unfolded form it replaces: the (B*T, cd+de) concat
of the code expansion and c_trg (AutoVC.py:197-204) fed to the LSTM layer (AutoVC.py:96,103).
Same h, and the same gradients for codes, c_trg and all four LSTM parameters.  fp32 compute:
the two forms differ only in fp32 summation order (rel 1e-5); bf16: both round the same
operands to bf16, the fold sums the 16 frames of a code in fp32 before the GEMM (rel 2e-2)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _relf(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


@pytest.mark.parametrize("comp,B,T,nc,tol", [("fp32", 3, 32, 2, 1e-5), ("bf16", 8, 64, 4, 2e-2),
                                              ("bf16", 64, 128, 8, 2e-2)])
def test_lstm1_fold_matches_concat_path(comp, B, T, nc, tol):
    import autoformer_amd as A
    from autoformer_amd import layers as Lyr
    from autoformer_amd.factory.Norm import LSTMParams

    A.set_compute(comp)
    try:
        torch.manual_seed(0)
        cd, de, H = 88, 256, 512
        mod = LSTMParams(cd + de, H, 1, batch_first=True).to(DEV)
        core = Lyr.LSTMLayerCore(mod, 0)
        codes0 = torch.randn(B, nc * cd, device=DEV)
        emb0 = torch.randn(B, de, device=DEV)
        dh = torch.randn(B * T, H, device=DEV)
        outs = []
        for fold in (False, True):
            codes = codes0.clone().requires_grad_(True)
            emb = emb0.clone().requires_grad_(True)
            for p in mod.parameters():
                p.grad = None
            calls = []
            if fold:
                h = Lyr.lstm1_folded(mod, core, codes, emb, B, T, nc, cd, hook=lambda: calls.append(1))
            else:
                x = Lyr.dec_concat(codes, emb, B, T, nc, cd)
                h = Lyr.lstm(mod, [core], x, B, T)
            h.backward(dh)
            torch.cuda.synchronize()
            Lyr.join_side()
            if fold:
                assert calls == [1]
            outs.append([h.detach().clone(), codes.grad.clone(), emb.grad.clone()] +
                        [p.grad.clone() for p in core.params()])
        names = ["h", "dcodes", "dc_trg", "dW_ih", "dW_hh", "db_ih", "db_hh"]
        for n, a, b in zip(names, outs[1], outs[0]):
            assert _relf(a, b) < tol, (n, _relf(a, b))
    finally:
        A.set_compute("bf16")


@pytest.mark.parametrize("B,T,nc,H", [(64, 128, 8, 512), (3, 36, 4, 512), (20, 32, 1, 1024), (5, 12, 12, 768)])
def test_lstm_fold_kernels_match_expanded_launch(B, T, nc, H):
    """avc_lstm_fwd_fold reads row b*nc + t/(T/nc) of the per-code projection: bit-identical to the
    ordinary persistent launch on the expanded (B*T, 4H) rows.  avc_lstm_bwd_fold: the same bf16
    dG as avc_lstm_bwd, and the in-recurrence segment sums equal avc_segsum over its fp32 dG up to
    fp32 summation order (frames taken in reverse); the s_code twin is s_code rounded to bf16.
    Ragged batches (B = 3, 5, 20: partial groups of 8), one code (nc = 1) and one frame per code."""
    import autoformer_amd as A
    from autoformer_amd import kernels as Kr

    A.set_compute("bf16")
    G = 4 * H
    if not (Kr.lstm_persistent_fwd(B, H, 1) and Kr.lstm_persistent_bwd(B, H, 1)):
        pytest.skip("shape not on the persistent path on this device")
    g = torch.Generator(device=DEV).manual_seed(3)
    pcode = torch.randn(B * nc, G, device=DEV, generator=g) * 0.5
    whh = (torch.randn(G, H, device=DEV, generator=g) * H ** -0.5).bfloat16()
    whh_t = whh.t().contiguous()
    hb = Kr.lstm_scratch(B, H, 1, DEV)
    h1, c1, g1 = Kr.lstm_fwd_fold(pcode, nc, whh, B, T, H, hb)
    xproj = Kr.expand_codes(pcode, torch.zeros(B, G, device=DEV), B, T, nc)
    h0, c0, g0 = Kr.lstm_fwd(xproj, whh, B, T, H, 1, Kr.lstm_scratch(B, H, 1, DEV))
    torch.cuda.synchronize()
    assert Kr.lstm_timeout_flag(hb, B, H) == 0
    assert torch.equal(h1, h0) and torch.equal(c1, c0) and torch.equal(g1, g0)
    assert torch.equal(h1._bf16, h0._bf16)
    dh = torch.randn(B * T, H, device=DEV, generator=g)
    dg16, sc = Kr.lstm_bwd_fold(dh, c0, g0, whh_t, B, T, H, nc)
    dg = Kr.lstm_bwd(dh, h0, c0, g0, None, whh_t, B, T, H, 1)
    ref = Kr.segsum(dg, B * nc, T // nc, G, ld=G)
    torch.cuda.synchronize()
    assert torch.equal(dg16, dg._bf16)
    assert _relf(sc, ref) < 1e-6, _relf(sc, ref)
    assert torch.equal(sc._bf16, sc.bfloat16())
