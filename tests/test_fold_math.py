"""CPU check of the encoder conv0 fold's algebra (fold.hip, layers._EncConv0FoldFn) against
torch.nn.functional.conv1d on the concatenated input (reference factory/AutoVC.py:46-51):
the speaker half of the conv as an edge-class row bias (forward) and the per-tap column sums of
dy (weight and embedding gradients), with the kernels' index conventions restated in torch."""
import torch

from tests.capture_ref import edge_class, row_bias_rows


def _edge_table(E, B, Co, K, T, pad):
    # restatement of conv_edge_table_kernel: S[b][cls][co] = sum over valid taps of E[b][k][co]
    ncls = 2 * pad + 1
    S = torch.zeros(B, ncls, Co, dtype=E.dtype)
    for cls in range(ncls):
        t = cls if cls < pad else (pad if cls == pad else T - 1 - (2 * pad - cls))
        for k in range(K):
            if 0 <= t + k - pad < T:
                S[:, cls] += E.view(B, K, Co)[:, k]
    return S.view(B * ncls, Co)


def _edge_colsum(dy, B, T, C, K, pad):
    d = dy.view(B, T, C)
    out = torch.zeros(B, K, C, dtype=dy.dtype)
    for k in range(K):
        lo, hi = max(0, pad - k), min(T, T + pad - k)
        out[:, k] = d[:, lo:hi].sum(1)
    return out.view(B * K, C)


def test_fold_matches_concat_conv():
    torch.manual_seed(0)
    B, T, nm, de, Co, K, pad = 3, 11, 6, 5, 7, 5, 2
    mel = torch.randn(B, nm, T, dtype=torch.float64)
    emb = torch.randn(B, de, dtype=torch.float64, requires_grad=True)
    w = torch.randn(Co, nm + de, K, dtype=torch.float64, requires_grad=True)
    x = torch.cat([mel, emb[:, :, None].expand(B, de, T)], 1)
    y = torch.nn.functional.conv1d(x, w, padding=pad)  # (B, Co, T)
    # fold: conv over mel alone + row bias S[b][class(t)]
    We = w.detach()[:, nm:, :].permute(2, 0, 1).reshape(K * Co, de)  # mode 2: We[k][co][ci]
    E = emb.detach() @ We.t()  # (B, K*Co)
    S = _edge_table(E, B, Co, K, T, pad)
    ym = torch.nn.functional.conv1d(mel, w.detach()[:, :nm], padding=pad)
    yf = ym.transpose(1, 2).reshape(B * T, Co) + row_bias_rows(S, B * T, T, pad)
    assert (yf - y.detach().transpose(1, 2).reshape(B * T, Co)).abs().max() < 1e-10
    assert edge_class(T, pad).tolist() == [0, 1] + [2] * (T - 4) + [3, 4]
    # backward: weight gradient of the embedding half and the embedding gradient from Sdy
    dy = torch.randn(B, Co, T, dtype=torch.float64)
    y.backward(dy)
    dyf = dy.transpose(1, 2).reshape(B * T, Co)
    Sdy = _edge_colsum(dyf, B, T, Co, K, pad).view(B, K, Co)
    dWe = torch.einsum("bkc,bi->cik", Sdy, emb.detach())  # dW[co][nm + ci][k]
    assert (dWe - w.grad[:, nm:]).abs().max() < 1e-10
    demb = torch.einsum("bkc,kci->bi", Sdy, We.view(K, Co, de))
    assert (demb - emb.grad).abs().max() < 1e-10
