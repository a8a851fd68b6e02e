"""Per-kernel numerics on the MI355X, through the C-ABI, against plain PyTorch fp32
references of the same op (computed on the CPU).

Tolerances: fp32 compute (exact fp32 MFMA) -> rel <= 1e-5 (GEMM) / 1e-4 (recurrences);
bf16 compute -> rel-Frobenius <= 1.5e-2.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(autouse=True)
def _fp32():
    import autoformer_amd as A

    A.set_compute("fp32")
    torch.manual_seed(0)
    yield
    A.set_compute("fp32")


def relf(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return float((a - b).norm() / max(b.norm().item(), 1e-30))


def rinf(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return float((a - b).abs().max() / max(b.abs().max().item(), 1e-30))


def _gemm_ref(A_, B_):  # A (M,K) B (N,K)
    return A_.double() @ B_.double().t()


@pytest.mark.parametrize("M,N,K", [(300, 200, 96), (128, 128, 32), (7, 9, 20), (1000, 80, 400)])
@pytest.mark.parametrize("comp", ["fp32", "bf16"])
def test_gemm_plain_all_layouts(M, N, K, comp):
    import autoformer_amd as A
    from autoformer_amd import kernels as Kr

    A.set_compute(comp)
    a = torch.randn(M, K)
    b = torch.randn(N, K)
    ref = _gemm_ref(a, b)
    tol = 1e-5 if comp == "fp32" else 1.5e-2
    for aks in (False, True):
        for bks in (False, True):
            ad = (a.t().contiguous() if aks else a).to(DEV)
            bd = (b.t().contiguous() if bks else b).to(DEV)
            c = torch.empty(M, N, device=DEV)
            Kr.gemm(M, N, K, Kr.operand(ad, M if aks else K, kstrided=aks), Kr.operand(bd, N if bks else K, kstrided=bks), c)
            assert relf(c, ref) < tol, (aks, bks, relf(c, ref))


def test_gemm_bias_accumulate_splitk_batch():
    from autoformer_amd import kernels as Kr

    M, N, K = 256, 192, 4096
    a, b, bias = torch.randn(M, K), torch.randn(N, K), torch.randn(N)
    ref = _gemm_ref(a, b) + bias.double()
    ad, bd = a.to(DEV), b.to(DEV)
    for sk in (1, 4):
        c = torch.empty(M, N, device=DEV)
        Kr.gemm(M, N, K, Kr.operand(ad, K), Kr.operand(bd, K), c, bias=bias.to(DEV), split_k=sk)
        assert relf(c, ref) < 1e-5
    c0 = torch.randn(M, N)
    c = c0.to(DEV)
    Kr.gemm(M, N, K, Kr.operand(ad, K), Kr.operand(bd, K), c, accumulate=True, split_k=3)
    assert relf(c, ref - bias.double() + c0.double()) < 1e-5
    # batched: 3 independent products with per-batch A and C strides, shared B
    Bn = 3
    a3 = torch.randn(Bn, 64, 48)
    c3 = torch.empty(Bn, 64, 40, device=DEV)
    b3 = torch.randn(40, 48)
    Kr.gemm(64, 40, 48, Kr.operand(a3.to(DEV), 48, batch_stride=64 * 48), Kr.operand(b3.to(DEV), 48), c3, batch=Bn,
            c_batch_stride=64 * 40)
    assert relf(c3, torch.einsum("bmk,nk->bmn", a3.double(), b3.double())) < 1e-5


@pytest.mark.parametrize("B,T,Cin,Cout,Kw,pad", [(2, 176, 336, 512, 5, 2), (3, 37, 80, 96, 5, 2), (2, 80, 176, 88, 3, 0),
                                                  (2, 30, 44, 22, 3, 0), (4, 64, 512, 96, 5, 2), (3, 40, 64, 512, 5, 2)])
@pytest.mark.parametrize("comp", ["fp32", "bf16"])
def test_conv_gemm_fwd_dgrad_wgrad(B, T, Cin, Cout, Kw, pad, comp):
    """Conv1d as a windowed GEMM: forward, data- and weight-gradient vs F.conv1d autograd."""
    import autoformer_amd as A
    from autoformer_amd import kernels as Kr

    A.set_compute(comp)
    tol = 1e-5 if comp == "fp32" else 1.5e-2
    x = torch.randn(B, Cin, T, requires_grad=True)
    w = torch.randn(Cout, Cin, Kw, requires_grad=True) * 0.1
    w.retain_grad()
    y = F.conv1d(x, w, padding=pad)
    To = y.shape[-1]
    gy = torch.randn_like(y)
    y.backward(gy)
    dt = Kr.BF16 if comp == "bf16" else Kr.F32
    xf = x.detach().transpose(1, 2).reshape(B * T, Cin).contiguous().to(DEV)
    if comp == "bf16":  # bf16 activations: the forms the halo conv kernel (gemm_conv.hip) takes
        xf = xf.to(torch.bfloat16)
    wd = w.detach().to(DEV)
    Wf = Kr.conv_pack(wd, 0, dt)
    Wd = Kr.conv_pack(wd, 1, dt)
    out = torch.empty(B * To, Cout, device=DEV)
    Kr.gemm(B * To, Cout, Kw * Cin, Kr.operand(xf, Cin, window=(Kw, pad, To, T, Cin)), Kr.operand(Wf, Kw * Cin), out)
    assert relf(out, y.detach().transpose(1, 2).reshape(B * To, Cout)) < tol
    gyf = gy.transpose(1, 2).reshape(B * To, Cout).contiguous().to(DEV)
    if comp == "bf16":
        gyf = gyf.to(torch.bfloat16)
    dx = torch.empty(B * T, Cin, device=DEV)
    Kr.gemm(B * T, Cin, Kw * Cout, Kr.operand(gyf, Cout, window=(Kw, Kw - 1 - pad, T, To, Cout)),
            Kr.operand(Wd, Kw * Cout), dx)
    assert relf(dx, x.grad.transpose(1, 2).reshape(B * T, Cin)) < tol
    dwf = torch.empty(Cout, Kw * Cin, device=DEV)
    Kr.gemm(Cout, Kw * Cin, B * To, Kr.operand(gyf, Cout, kstrided=True),
            Kr.operand(xf, Cin, kstrided=True, window=(Kw, pad, To, T, Cin)), dwf, split_k=2)
    dw = Kr.conv_grad_unpack(dwf, Cout, Cin, Kw)
    assert relf(dw, w.grad) < tol


def test_gemm_time_shift_window():
    """k-strided frame window with taps=1 (the LSTM h_{t-1} / h_{t+1} shift)."""
    from autoformer_amd import kernels as Kr

    B, T, H, G = 3, 20, 44, 176
    dg = torch.randn(B * T, G)
    h = torch.randn(B, T, H)
    for shift, ref_h in ((1, torch.cat([torch.zeros(B, 1, H), h[:, :-1]], 1)),
                         (-1, torch.cat([h[:, 1:], torch.zeros(B, 1, H)], 1))):
        out = torch.empty(G, H, device=DEV)
        Kr.gemm(G, H, B * T, Kr.operand(dg.to(DEV), G, kstrided=True),
                Kr.operand(h.reshape(B * T, H).to(DEV), H, kstrided=True, window=(1, shift, T, T, H)), out)
        ref = dg.double().t() @ ref_h.reshape(B * T, H).double()
        assert relf(out, ref) < 1e-5


@pytest.mark.parametrize("M,C", [(8192, 512), (352, 80), (300, 176)])
def test_bn_stats_epilogue_and_finalize(M, C):
    from autoformer_amd import kernels as Kr

    x = torch.randn(M, 64) * 3
    w = torch.randn(C, 64)
    y = x.double() @ w.double().t() + 5.0  # large mean: checks the centred (Chan) merge
    bias = torch.full((C,), 5.0)
    yd = torch.empty(M, C, device=DEV)
    part = Kr.bn_partial_buffer(M, C, DEV)
    Kr.gemm(M, C, 64, Kr.operand(x.to(DEV), 64), Kr.operand(w.to(DEV), 64), yd, bias=bias.to(DEV), bn_partial=part)
    gamma, beta = torch.rand(C) + 0.5, torch.randn(C)
    rm, rv, nbt = torch.randn(C).to(DEV), (torch.rand(C) + 0.5).to(DEV), torch.zeros((), dtype=torch.long, device=DEV)
    rm0, rv0 = rm.cpu().double(), rv.cpu().double()
    mean, rstd, scale, shift = Kr.bn_finalize(part, M, C, gamma.to(DEV), beta.to(DEV), rm, rv, nbt, 0.1, 1e-5)
    m_ref = y.mean(0)
    v_ref = y.var(0, unbiased=False)
    assert rinf(mean, m_ref) < 1e-5
    assert rinf(rstd, 1 / torch.sqrt(v_ref + 1e-5)) < 1e-4
    assert rinf(rm, 0.9 * rm0 + 0.1 * m_ref) < 1e-5
    assert rinf(rv, 0.9 * rv0 + 0.1 * y.var(0, unbiased=True)) < 1e-4
    assert int(nbt.item()) == 1


@pytest.mark.parametrize("M,C,ld", [(4864, 44, 44), (4736, 22, 22), (300, 70, 80), (77, 5, 8), (128, 512, 512)])
def test_bn_stats_plain(M, C, ld):
    """avc_bn_stats (the stats pass for activations no GEMM produced: the Discriminator's BNs)
    + finalize against fp64 batch statistics, ragged row tiles and a row stride > C."""
    from autoformer_amd import kernels as Kr

    y = torch.randn(M, ld) * 2 + 3.0
    yd = y.to(DEV)
    part = Kr.bn_stats(yd, M, C, ld=ld)
    mean, rstd, _, _ = Kr.bn_finalize(part, M, C, None, None, None, None, None, 0.1, 1e-5)
    ref = y[:, :C].double()
    assert rinf(mean, ref.mean(0)) < 1e-5
    assert rinf(rstd, 1 / torch.sqrt(ref.var(0, unbiased=False) + 1e-5)) < 1e-4


@pytest.mark.parametrize("M,C,Kd", [(8192, 512, 2560), (352, 80, 64), (300, 176, 64), (1000, 1024, 128)])
@pytest.mark.parametrize("comp,nupd", [("bf16", 1), ("bf16", 2), ("fp32", 2)])
def test_gemm_bn_fused_finalize(M, C, Kd, comp, nupd):
    """avc_gemm_bn: the BN finalize done by the GEMM's last-arriving row tile of each column tile
    (bf16 fast kernels) or by finalize launches after it (fp32 generic kernel) == the separate
    avc_bn_finalize on the same partials; running statistics updated nupd times."""
    import autoformer_amd as A
    from autoformer_amd import kernels as Kr

    A.set_compute(comp)
    try:
        x = (torch.randn(M, Kd, device=DEV) * 3)
        w = torch.randn(C, Kd, device=DEV)
        bias = torch.full((C,), 5.0, device=DEV)
        gamma, beta = (torch.rand(C) + 0.5).to(DEV), torch.randn(C).to(DEV)
        rm0, rv0 = torch.randn(C).to(DEV), (torch.rand(C) + 0.5).to(DEV)
        y1 = torch.empty(M, C, device=DEV)
        p1 = Kr.bn_partial_buffer(M, C, DEV)
        rm1, rv1, n1 = rm0.clone(), rv0.clone(), torch.zeros((), dtype=torch.long, device=DEV)
        st1 = Kr.gemm(M, C, Kd, Kr.operand(x, Kd), Kr.operand(w, Kd), y1, bias=bias, bn_partial=p1,
                      bn_fin=(gamma, beta, rm1, rv1, n1, 0.1, 1e-5, nupd))
        y2 = torch.empty(M, C, device=DEV)
        p2 = Kr.bn_partial_buffer(M, C, DEV)
        rm2, rv2, n2 = rm0.clone(), rv0.clone(), torch.zeros((), dtype=torch.long, device=DEV)
        Kr.gemm(M, C, Kd, Kr.operand(x, Kd), Kr.operand(w, Kd), y2, bias=bias, bn_partial=p2)
        for _ in range(nupd):
            st2 = Kr.bn_finalize(p2, M, C, gamma, beta, rm2, rv2, n2, 0.1, 1e-5)
        assert torch.equal(y1, y2) and torch.equal(p1, p2)
        for a, b in zip(st1, st2):
            assert rinf(a, b) < 1e-6
        assert rinf(rm1, rm2) < 1e-6 and rinf(rv1, rv2) < 1e-6
        assert int(n1.item()) == nupd == int(n2.item())
        yf = y2.double().cpu()
        assert rinf(st1[0], yf.mean(0)) < 1e-5
        assert rinf(st1[1], 1 / torch.sqrt(yf.var(0, unbiased=False) + 1e-5)) < 1e-4
    finally:
        A.set_compute("bf16")


@pytest.mark.parametrize("act", [0, 1, 2])
@pytest.mark.parametrize("from_pre", [False, True])
@pytest.mark.parametrize("M,C", [(1000, 96), (1000, 90), (8192, 512), (300, 80)])
def test_bn_act_forward_backward(act, from_pre, M, C):
    """BN + activation backward; from_pre: act' recomputed from yhat*gamma + beta (a = None),
    C = 90 takes the scalar (C % 4 != 0) kernels, the others the fused reduce/apply pair."""
    from autoformer_amd import kernels as Kr

    y = torch.randn(M, C) * 2 + 1
    gamma, beta = torch.rand(C) + 0.5, torch.randn(C)
    yt = y.clone().requires_grad_(True)
    g_t = gamma.clone().requires_grad_(True)
    b_t = beta.clone().requires_grad_(True)
    z = F.batch_norm(yt.t().unsqueeze(0), None, None, g_t, b_t, True, 0.1, 1e-5).squeeze(0).t()
    a_ref = [z, torch.relu(z), torch.tanh(z)][act]
    dA = torch.randn(M, C)
    a_ref.backward(dA)
    yd = y.to(DEV)
    part = Kr.bn_stats(yd, M, C)
    mean, rstd, scale, shift = Kr.bn_finalize(part, M, C, gamma.to(DEV), beta.to(DEV), None, None, None, 0.1, 1e-5)
    a = Kr.bn_apply(yd, scale, shift, act)
    assert rinf(a, a_ref.detach()) < 1e-5
    if from_pre:
        dy, dgam, dbet, dbias = Kr.bn_bwd(dA.to(DEV), None, yd, mean, rstd, gamma.to(DEV), act, beta=beta.to(DEV))
    else:
        dy, dgam, dbet, dbias = Kr.bn_bwd(dA.to(DEV), a, yd, mean, rstd, gamma.to(DEV), act)
    assert relf(dy, yt.grad) < 1e-4
    assert relf(dgam, g_t.grad) < 1e-5
    assert relf(dbet, b_t.grad) < 1e-5
    assert float(dbias.abs().max()) < 1e-3


@pytest.mark.parametrize("act", [1, 2])
@pytest.mark.parametrize("M,C", [(8192, 512), (1000, 90), (300, 80)])
def test_bn_bf16_storage(act, M, C):
    """bf16-stored y / dA / outputs (bf16 compute mode): the kernels compute in fp32 from the
    bf16 values, so they must match the fp32 path run on the same bf16-rounded inputs to fp32
    rounding, and the bf16-only outputs must be those results rounded once."""
    from autoformer_amd import kernels as Kr

    y = (torch.randn(M, C) * 2 + 1).bfloat16()
    dA = torch.randn(M, C).bfloat16()
    gamma, beta = torch.rand(C) + 0.5, torch.randn(C)
    yd, y32 = y.to(DEV), y.float().to(DEV)
    part = Kr.bn_stats(y32, M, C)
    mean, rstd, scale, shift = Kr.bn_finalize(part, M, C, gamma.to(DEV), beta.to(DEV), None, None, None, 0.1, 1e-5)
    a32 = Kr.bn_apply(y32, scale, shift, act)
    a16 = Kr.bn_apply(yd, scale, shift, act, out_bf16=True)
    assert a16.dtype == torch.bfloat16
    assert torch.equal(a16, a32.bfloat16())
    g_, b_ = gamma.to(DEV), beta.to(DEV)
    dy32, dg32, db32, _ = Kr.bn_bwd(dA.float().to(DEV), None, y32, mean, rstd, g_, act, beta=b_)
    dy16, dg16, db16, _ = Kr.bn_bwd(dA.to(DEV), None, yd, mean, rstd, g_, act, beta=b_, dy_bf16=True)
    assert dy16.dtype == torch.bfloat16
    assert torch.equal(dy16, dy32.bfloat16())
    assert torch.equal(dg16, dg32) and torch.equal(db16, db32)


def test_gemm_bf16_only_output():
    """c dtype bf16: the epilogue stores only the bf16 rounding of the fp32 result (with bias
    and BN partial statistics taken from the fp32 accumulators)."""
    import autoformer_amd as A
    from autoformer_amd import kernels as Kr

    A.set_compute("bf16")
    M, N, Kd = 1024, 512, 320
    x = torch.randn(M, Kd, device=DEV).bfloat16()
    w = torch.randn(N, Kd, device=DEV).bfloat16()
    bias = torch.randn(N, device=DEV)
    c32 = torch.empty(M, N, device=DEV)
    p32 = Kr.bn_partial_buffer(M, N, DEV)
    Kr.gemm(M, N, Kd, Kr.operand(x, Kd), Kr.operand(w, Kd), c32, bias=bias, bn_partial=p32)
    c16 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    p16 = Kr.bn_partial_buffer(M, N, DEV)
    Kr.gemm(M, N, Kd, Kr.operand(x, Kd), Kr.operand(w, Kd), c16, bias=bias, bn_partial=p16)
    assert torch.equal(c16, c32.bfloat16())
    assert torch.equal(p16, p32)


def _lstm_case(B, T, In, H, dirs, comp):
    import autoformer_amd as A
    from autoformer_amd import kernels as Kr
    from autoformer_amd.factory.Norm import LSTMParams
    from autoformer_amd.layers import LSTMLayerCore, lstm

    A.set_compute(comp)
    mod = LSTMParams(In, H, 1, bidirectional=dirs == 2)
    x = torch.randn(B, T, In)
    ref_mod = torch.nn.LSTM(In, H, 1, batch_first=True, bidirectional=dirs == 2)
    ref_mod.load_state_dict(mod.state_dict())
    xr = x.clone().requires_grad_(True)
    out_ref, _ = ref_mod(xr)
    gy = torch.randn_like(out_ref)
    out_ref.backward(gy)
    mod = mod.to(DEV)
    xd = x.reshape(B * T, In).to(DEV).requires_grad_(True)
    core = LSTMLayerCore(mod, 0)
    out = lstm(mod, [core], xd, B, T)
    out.backward(gy.reshape(B * T, -1).to(DEV))
    torch.cuda.synchronize()
    res = {"out": relf(out.detach(), out_ref.detach().reshape(B * T, -1)),
           "dx": relf(xd.grad, xr.grad.reshape(B * T, In))}
    for (n, p), (n2, p2) in zip(mod.named_parameters(), ref_mod.named_parameters()):
        assert n == n2
        res[n] = relf(p.grad, p2.grad)
    return res


@pytest.mark.parametrize("B,T,In,H,dirs", [(4, 33, 512, 44, 2), (3, 20, 88, 44, 2), (5, 17, 344, 512, 1),
                                           (20, 9, 512, 1024, 1), (2, 12, 96, 128, 2), (2, 176, 96, 64, 1),
                                           (3, 50, 40, 16, 2)])
def test_lstm_layer_fp32(B, T, In, H, dirs):
    res = _lstm_case(B, T, In, H, dirs, "fp32")
    bad = {k: v for k, v in res.items() if v > 1e-4}
    assert not bad, bad


@pytest.mark.parametrize("B,T,In,H,dirs", [(4, 33, 512, 44, 2), (20, 16, 512, 1024, 1), (64, 8, 344, 512, 1)])
def test_lstm_layer_bf16(B, T, In, H, dirs):
    res = _lstm_case(B, T, In, H, dirs, "bf16")
    bad = {k: v for k, v in res.items() if v > 3e-2}
    assert not bad, bad


def test_glue_kernels():
    from autoformer_amd import kernels as Kr

    B, T, D, freq = 3, 32, 44, 8
    lo = torch.randn(B, T, 2 * D)
    codes = Kr.codes_gather(lo.reshape(B * T, 2 * D).to(DEV), B, T, D, freq)
    ref = torch.cat([torch.cat((lo[:, i + freq - 1, :D], lo[:, i, D:]), -1) for i in range(0, T, freq)], -1)
    assert rinf(codes, ref) == 0.0
    dc = torch.randn(B, (T // freq) * 2 * D)
    lo_r = lo.clone().requires_grad_(True)
    ref2 = torch.cat([torch.cat((lo_r[:, i + freq - 1, :D], lo_r[:, i, D:]), -1) for i in range(0, T, freq)], -1)
    ref2.backward(dc)
    dlo = Kr.codes_scatter(dc.to(DEV), B, T, D, freq)
    assert rinf(dlo, lo_r.grad.reshape(B * T, 2 * D)) == 0.0
    emb = torch.randn(B, 256)
    out = Kr.dec_concat(codes, emb.to(DEV), B, T, T // freq, 2 * D)
    cl = list(ref.split(2 * D, -1))
    ref3 = torch.cat((torch.cat([c.unsqueeze(1).expand(-1, freq, -1) for c in cl], 1),
                      emb.unsqueeze(1).expand(-1, T, -1)), -1)
    assert rinf(out, ref3.reshape(B * T, -1)) == 0.0
    mel = torch.randn(B, T, 80)
    xc = Kr.enc_concat(mel.reshape(B * T, 80).to(DEV), emb.to(DEV), B, T)
    assert rinf(xc, torch.cat((mel, emb.unsqueeze(1).expand(-1, T, -1)), -1).reshape(B * T, -1)) == 0.0


def test_losses_and_adam():
    from autoformer_amd import kernels as Kr

    a, b = torch.randn(5000), torch.randn(5000)
    ad, bd = a.to(DEV), b.to(DEV)
    assert abs(Kr.mse_loss(ad, bd).item() - F.mse_loss(a, b).item()) < 1e-5
    assert abs(Kr.l1_loss(ad, bd).item() - F.l1_loss(a, b).item()) < 1e-5
    # Adam vs torch.optim.Adam for 3 steps
    p = torch.randn(1000)
    pt = p.clone().requires_grad_(True)
    opt = torch.optim.Adam([pt], 1e-3)
    pd, m, v = p.to(DEV), torch.zeros(1000, device=DEV), torch.zeros(1000, device=DEV)
    st = torch.zeros(4, device=DEV)
    for i in range(3):
        g = torch.randn(1000)
        pt.grad = g.clone()
        opt.step()
        Kr.adam(pd, g.to(DEV), m, v, 1e-3, 0.9, 0.999, 1e-8, st)
    assert rinf(pd, pt.detach()) < 1e-6


def test_gemm_fast_bf16_copy_and_mixed_dtypes():
    import autoformer_amd as A
    from autoformer_amd import kernels as Kr

    A.set_compute("bf16")
    M, N, K_ = 512, 320, 256
    a = torch.randn(M, K_)
    b = torch.randn(N, K_)
    ref = _gemm_ref(a.bfloat16().float(), b.bfloat16().float())
    for adt in (torch.float32, torch.bfloat16):
        for bdt in (torch.float32, torch.bfloat16):
            ad, bd = a.to(DEV).to(adt), b.to(DEV).to(bdt)
            c = torch.empty(M, N, device=DEV)
            c16 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            Kr.gemm(M, N, K_, Kr.operand(ad, K_), Kr.operand(bd, K_), c, c_bf16=c16)
            assert relf(c, ref) < 1e-5
            assert relf(c16.float(), ref) < 5e-3


@pytest.mark.parametrize("B,H", [(64, 1024), (20, 1024), (64, 512), (3, 512), (64, 768), (2, 768)])
def test_lstm_persistent_forward_matches_per_step(B, H):
    """The persistent recurrence (bf16) equals the per-step kernels within bf16 rounding and
    never raises its spin-timeout flag."""
    import os
    import autoformer_amd as A
    from autoformer_amd import kernels as Kr
    from autoformer_amd import _lib

    A.set_compute("bf16")
    T = 37
    G = 4 * H
    torch.manual_seed(1)
    xproj = (torch.randn(B * T, G) * 0.5).to(DEV)
    whh = (torch.randn(G, H) * (1.0 / H ** 0.5)).to(DEV).bfloat16()
    hb = Kr.lstm_scratch(B, H, 1, DEV)
    h1, c1, g1 = Kr.lstm_fwd(xproj, whh, B, T, H, 1, hb)
    torch.cuda.synchronize()
    assert Kr.lstm_timeout_flag(hb, B, H) == 0
    # reference: fp32 loop on the CPU with the same (bf16-rounded) weights, h rounded to bf16
    w = whh.float().cpu()
    xp = xproj.cpu().view(B, T, G)
    h = torch.zeros(B, H)
    c = torch.zeros(B, H)
    outs = []
    for t in range(T):
        gts = xp[:, t] + h.bfloat16().float() @ w.t()
        i, f, gg, o = gts.chunk(4, 1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
        h = torch.sigmoid(o) * torch.tanh(c)
        outs.append(h)
    ref = torch.stack(outs, 1).reshape(B * T, H)
    assert relf(h1, ref) < 2e-3, relf(h1, ref)
    assert relf(c1.cpu().view(B, T, H)[:, -1], c) < 2e-3


@pytest.mark.parametrize("M,N,K,split", [(300, 200, 96, 1), (1000, 80, 400, 1), (1024, 512, 2560, 1),
                                         (513, 640, 1024, 3), (64, 136, 8, 1)])
def test_gemm_nt_lds_pipeline_bf16_operands(M, N, K, split):
    """bf16 K-contiguous operands take the LDS-DMA NT kernel (gemm_nt.hip): products of bf16
    values accumulate in fp32, so the result matches an fp64 product of the same bf16 values
    to fp32 accumulation error (M/N tails, K tails of 8, split-K, bias)."""
    import autoformer_amd as A
    from autoformer_amd import kernels as Kr

    A.set_compute("bf16")
    a = torch.randn(M, K).to(torch.bfloat16)
    b = torch.randn(N, K).to(torch.bfloat16)
    bias = torch.randn(N)
    ref = _gemm_ref(a.float(), b.float()) + bias.double()
    c = torch.empty(M, N, device=DEV)
    ad, bd = a.to(DEV), b.to(DEV)
    Kr.gemm(M, N, K, Kr.operand(ad, K), Kr.operand(bd, K), c, bias=bias.to(DEV), split_k=split)
    assert relf(c, ref) < 1e-5, relf(c, ref)


@pytest.mark.parametrize("B,T,Cin,Cout,Kw,pad", [(3, 37, 64, 96, 5, 2), (64, 128, 512, 512, 5, 2), (2, 9, 8, 24, 3, 1),
                                                 (8, 176, 512, 80, 5, 2), (5, 50, 96, 136, 5, 2), (1, 3, 32, 64, 5, 2)])
def test_gemm_nt_conv_window_and_bn_stats(B, T, Cin, Cout, Kw, pad):
    """Windowed (im2col) A operand + the BN partial-statistics epilogue.  Five-tap 'same' convs
    with Cin % 32 == 0 take the halo-reuse conv kernel (gemm_conv.hip): tiles inside one
    utterance (T=128), tiles spanning utterances (T=37, 50, 176), utterances shorter than the
    halo (T=3), and output-channel tails (80, 96, 136)."""
    import autoformer_amd as A
    from autoformer_amd import kernels as Kr

    A.set_compute("bf16")
    x = torch.randn(B, T, Cin).to(torch.bfloat16)
    w = (torch.randn(Cout, Cin, Kw) * 0.1).to(torch.bfloat16)
    ref = F.conv1d(x.float().transpose(1, 2).double(), w.float().double(), padding=pad).transpose(1, 2)
    ref = ref.reshape(B * T, Cout)
    Wf = w.permute(0, 2, 1).reshape(Cout, Kw * Cin).contiguous().to(DEV)  # [co][k][ci]
    M = B * T
    y = torch.empty(M, Cout, device=DEV)
    part = Kr.bn_partial_buffer(M, Cout, DEV)
    Kr.gemm(M, Cout, Kw * Cin, Kr.operand(x.reshape(M, Cin).to(DEV), Cin, window=(Kw, pad, T, T, Cin)),
            Kr.operand(Wf, Kw * Cin), y, bn_partial=part)
    assert relf(y, ref) < 1e-5, relf(y, ref)
    mean, rstd, _, _ = Kr.bn_finalize(part, M, Cout, None, None, None, None, None, 0.1, 1e-5)
    refm = ref.mean(0)
    refv = ref.var(0, unbiased=False)
    assert rinf(mean, refm) < 1e-4
    assert rinf(1.0 / rstd.double() ** 2 - 1e-5, refv) < 1e-3


@pytest.mark.parametrize("B,H", [(64, 1024), (20, 1024), (64, 512), (3, 512), (64, 768), (2, 768)])
def test_lstm_persistent_backward(B, H):
    """The one-launch backward recurrence (bf16 products, fp32 cell math) against an fp32
    CPU loop that rounds dG_{t+1} to bf16 for the recurrent product, as the kernel does;
    its bf16 dG twin equals the fp32 output rounded; the spin-timeout flag stays clear."""
    import autoformer_amd as A

    A.set_compute("bf16")
    _persistent_backward_case(B, H)


def test_lstm_persistent_backward_under_load():
    """The hand-off under uneven load: the same backward run alone and beside a stream of large
    GEMMs on another stream (so members start and run at different times, and the payload lines
    compete with streaming traffic) is bit-identical -- the recurrence's arithmetic order is
    fixed, so any stale or torn payload read would show as a difference."""
    import autoformer_amd as A
    from autoformer_amd import kernels as Kr

    A.set_compute("bf16")
    B, H, T = 64, 1024, 48
    G = 4 * H
    torch.manual_seed(5)
    dh = (torch.randn(B * T, H) * 0.1).to(DEV)
    c = (torch.randn(B * T, H) * 0.7).to(DEV)
    gates = torch.rand(B * T, G) * 0.9 + 0.05
    gates[:, 2 * H:3 * H] = gates[:, 2 * H:3 * H] * 2 - 1
    gates = gates.to(DEV)
    wt = ((torch.randn(G, H) * (1.0 / H ** 0.5)).bfloat16().t().contiguous()).to(DEV)
    gbuf = Kr.lstm_bwd_scratch(B, H, 1, DEV)
    quiet = Kr.lstm_bwd(dh, dh, c, gates, None, wt, B, T, H, 1, gbuf=gbuf)
    torch.cuda.synchronize()
    assert Kr.lstm_bwd_timeout_flag(gbuf, B, H) == 0
    side = torch.cuda.Stream()
    x = torch.randn(4096, 4096, device=DEV, dtype=torch.bfloat16)
    for lead in (0, 1, 3):
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(lead):
                x = (x @ x).clamp_(-1, 1)
        loaded = Kr.lstm_bwd(dh, dh, c, gates, None, wt, B, T, H, 1, gbuf=gbuf)
        with torch.cuda.stream(side):
            for _ in range(4):
                x = (x @ x).clamp_(-1, 1)
        torch.cuda.synchronize()
        assert Kr.lstm_bwd_timeout_flag(gbuf, B, H) == 0
        assert torch.equal(loaded, quiet), (lead, (loaded - quiet).abs().max().item())
        assert torch.equal(loaded._bf16, quiet._bf16), lead


def _persistent_backward_case(B, H):
    from autoformer_amd import kernels as Kr

    assert Kr.lstm_persistent_bwd(B, H, 1)
    T = 29
    G = 4 * H
    torch.manual_seed(2)
    dh = (torch.randn(B * T, H) * 0.1)
    c = torch.randn(B * T, H) * 0.7
    gates = torch.rand(B * T, G) * 0.9 + 0.05
    gates[:, 2 * H:3 * H] = gates[:, 2 * H:3 * H] * 2 - 1  # g gate in (-1, 1)
    whh = (torch.randn(G, H) * (1.0 / H ** 0.5)).bfloat16()
    wt = whh.t().contiguous()
    gbuf = Kr.lstm_bwd_scratch(B, H, 1, DEV)
    dg = Kr.lstm_bwd(dh.to(DEV), dh.to(DEV), c.to(DEV), gates.to(DEV), None, wt.to(DEV), B, T, H, 1, gbuf=gbuf)
    torch.cuda.synchronize()
    assert Kr.lstm_bwd_timeout_flag(gbuf, B, H) == 0
    assert getattr(dg, "_bf16", None) is not None
    torch.testing.assert_close(dg._bf16.float(), dg.to(torch.bfloat16).float(), rtol=0, atol=0)
    w = whh.float()
    dhv, cv, gv = dh.view(B, T, H), c.view(B, T, H), gates.view(B, T, G)
    ref = torch.zeros(B, T, G)
    dc = torch.zeros(B, H)
    nxt = None
    for t in range(T - 1, -1, -1):
        d = dhv[:, t] + (nxt.bfloat16().float() @ w if nxt is not None else 0)
        i, f, gg, o = gv[:, t].chunk(4, 1)
        tc = torch.tanh(cv[:, t])
        cp = cv[:, t - 1] if t > 0 else torch.zeros(B, H)
        dcs = dc + d * o * (1 - tc * tc)
        out = torch.cat([dcs * gg * i * (1 - i), dcs * cp * f * (1 - f), dcs * i * (1 - gg * gg), d * tc * o * (1 - o)], 1)
        ref[:, t] = out
        dc = dcs * f
        nxt = out
    assert relf(dg, ref.reshape(B * T, G)) < 2e-3, relf(dg, ref.reshape(B * T, G))


def _im2col(x, B, T, Cin, Kw, pad):
    """(B*T, Cin) frames -> (B*T, Kw*Cin) window rows [tap][ci], zero outside each utterance."""
    xb = x.view(B, T, Cin)
    cols = torch.zeros(B, T, Kw, Cin, dtype=x.dtype)
    for k in range(Kw):
        src = torch.arange(T) + k - pad
        ok = (src >= 0) & (src < T)
        cols[:, ok, k] = xb[:, src[ok]]
    return cols.reshape(B * T, Kw * Cin)


@pytest.mark.parametrize("M,N,K,split", [(256, 640, 1000, 1), (80, 1024, 513, 3), (512, 2560, 2048, 2)])
def test_gemm_tt_lds_transposed_reads(M, N, K, split):
    """K-strided bf16 operands take the LDS-DMA TT kernel (gemm_tt.hip, ds_read_b64_tr_b16
    fragments); exact products of bf16 values, fp32 accumulation."""
    import autoformer_amd as A
    from autoformer_amd import kernels as Kr

    A.set_compute("bf16")
    a = torch.randn(K, M).to(torch.bfloat16)   # A[k][m]
    b = torch.randn(K, N).to(torch.bfloat16)   # B[k][n]
    ref = a.double().t() @ b.double()
    c = torch.empty(M, N, device=DEV)
    Kr.gemm(M, N, K, Kr.operand(a.to(DEV), M, kstrided=True), Kr.operand(b.to(DEV), N, kstrided=True), c,
            split_k=split)
    assert relf(c, ref) < 1e-5, relf(c, ref)


@pytest.mark.parametrize("B,T,Cin,Cout,Kw,pad", [(4, 37, 64, 96, 5, 2), (64, 128, 512, 512, 5, 2), (3, 20, 88, 176, 3, 1),
                                                 (3, 64, 96, 80, 5, 2), (2, 192, 32, 200, 5, 2),
                                                 (64, 176, 512, 512, 5, 2), (3, 100, 32, 80, 5, 2)])
@pytest.mark.parametrize("split", ["auto", 1])
def test_gemm_tt_conv_weight_gradient_window(B, T, Cin, Cout, Kw, pad, split):
    """Conv dW through the TT kernel.  5-tap 'same' convs with Cin % 32 == 0 take the halo form
    (one x tile for all taps; utterance edges zero-filled at load; K-tiles on the utterance grid,
    the last one of an utterance partial when T % 64 != 0: T = 37, 100, 176), the others the
    window stream; split-K (atomics) and single-pass (plain stores) epilogues."""
    import autoformer_amd as A
    from autoformer_amd import kernels as Kr

    A.set_compute("bf16")
    x = torch.randn(B * T, Cin).to(torch.bfloat16)
    dy = torch.randn(B * T, Cout).to(torch.bfloat16)
    ref = dy.double().t() @ _im2col(x.double(), B, T, Cin, Kw, pad)
    M, N = Cout, Kw * Cin
    c = torch.empty(M, N, device=DEV)
    Kr.gemm(M, N, B * T, Kr.operand(dy.to(DEV), Cout, kstrided=True),
            Kr.operand(x.to(DEV), Cin, kstrided=True, window=(Kw, pad, T, T, Cin)), c,
            split_k=Kr.auto_split_k(M, N, B * T) if split == "auto" else split)
    assert relf(c, ref) < 1e-5, relf(c, ref)


@pytest.mark.parametrize("kind", ["tt", "halo", "halo-cperm"])
def test_gemm_tt_splitk_reduction_accumulates_and_is_deterministic(kind):
    """Split-K TT products reduce their partials without atomics (gemm_internal.h splitk_last: the
    last-arriving split adds the write-through partial tiles in split order): accumulate=True adds
    the sum to C, and repeated launches are bit-identical (the atomics were not)."""
    import autoformer_amd as A
    from autoformer_amd import kernels as Kr

    A.set_compute("bf16")
    g = torch.Generator().manual_seed(11)
    if kind == "tt":
        M, N, K = 384, 640, 4096
        a = torch.randn(K, M, generator=g).to(torch.bfloat16)
        b = torch.randn(K, N, generator=g).to(torch.bfloat16)
        ref = a.double().t() @ b.double()
        opa, opb = Kr.operand(a.to(DEV), M, kstrided=True), Kr.operand(b.to(DEV), N, kstrided=True)
    else:
        B, T, Cin, M = 32, 128, 128, 256
        N, K = 5 * Cin, B * T
        x = torch.randn(B * T, Cin, generator=g).to(torch.bfloat16)
        dy = torch.randn(B * T, M, generator=g).to(torch.bfloat16)
        ref = dy.double().t() @ _im2col(x.double(), B, T, Cin, 5, 2)
        if kind == "halo-cperm":  # columns (tap, ci) stored in nn.Conv1d's [Co][Ci][K] order
            ref = ref.view(M, 5, Cin).transpose(1, 2).reshape(M, N)
        opa = Kr.operand(dy.to(DEV), M, kstrided=True)
        opb = Kr.operand(x.to(DEV), Cin, kstrided=True, window=(5, 2, T, T, Cin))
    base = torch.randn(M, N, generator=g)
    outs = []
    for split in (5, 5, 7, 1):
        c = base.to(DEV).clone()
        Kr.gemm(M, N, K, opa, opb, c, accumulate=True, split_k=split, cperm=5 if kind == "halo-cperm" else 0)
        torch.cuda.synchronize()
        outs.append(c.cpu())
        assert relf(c - base.to(DEV), ref) < 1e-5, relf(c - base.to(DEV), ref)
    assert torch.equal(outs[0], outs[1])


def test_gemm_tt_time_shift_window():
    """dW_hh = dG^T . h_{t-1}: B operand is h shifted one frame inside each utterance."""
    import autoformer_amd as A
    from autoformer_amd import kernels as Kr

    A.set_compute("bf16")
    B, T, H = 6, 23, 128
    G = 4 * H
    dg = torch.randn(B * T, G).to(torch.bfloat16)
    h = torch.randn(B * T, H).to(torch.bfloat16)
    hp = torch.zeros(B, T, H, dtype=torch.float64)
    hp[:, 1:] = h.double().view(B, T, H)[:, :-1]
    ref = dg.double().t() @ hp.reshape(B * T, H)
    c = torch.empty(G, H, device=DEV)
    Kr.gemm(G, H, B * T, Kr.operand(dg.to(DEV), G, kstrided=True),
            Kr.operand(h.to(DEV), H, kstrided=True, window=(1, 1, T, T, H)), c)
    assert relf(c, ref) < 1e-5, relf(c, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("Co,Ci,Kw", [(512, 512, 5), (96, 40, 5), (80, 512, 5), (512, 80, 5), (33, 65, 3), (24, 44, 9)])
def test_conv_pack_matches_permute(Co, Ci, Kw):
    """avc_conv_pack (LDS-staged tiles for <= 8 taps, the per-element kernel above) against the torch
    permutations it stands for: Wf[co][k][ci] and the flipped Wd[ci][K-1-k][co], bf16 and fp32."""
    from autoformer_amd import kernels as Kr

    w = torch.randn(Co, Ci, Kw, device=DEV)
    for dt, tdt in ((Kr.BF16, torch.bfloat16), (Kr.F32, torch.float32)):
        wf = Kr.conv_pack(w, 0, dt)
        wd = Kr.conv_pack(w, 1, dt)
        torch.cuda.synchronize()
        assert torch.equal(wf.reshape(Co, Kw, Ci), w.permute(0, 2, 1).to(tdt))
        assert torch.equal(wd.reshape(Ci, Kw, Co), w.flip(2).permute(1, 2, 0).to(tdt))


@pytest.mark.gpu
@pytest.mark.parametrize("Co,Ci,G,In,H", [(96, 40, 176, 72, 44), (512, 512, 4096, 1024, 1024), (33, 70, 130, 67, 33)])
def test_pack_batch_matches_individual_packs(Co, Ci, G, In, H):
    """avc_pack_batch (one launch for many packs) == the per-pack kernels it replaces, on ragged shapes too
    (tails of the 64 x 64 transpose tiles, the 4096-element copy units and the conv tiles; odd sizes take
    the unaligned scalar forms), the conv0 fold's channel-slice packs in all four layouts included."""
    import autoformer_amd as A
    from autoformer_amd import kernels as Kr
    from autoformer_amd import layers as Lyr

    A.set_compute("bf16")
    dev = "cuda:0"
    w = torch.randn(Co, Ci, 5, device=dev)
    wih, whh = torch.randn(G, In, device=dev), torch.randn(G, H, device=dev)
    bih, bhh = torch.randn(G, device=dev), torch.randn(G, device=dev)
    # the conv0 fold's channel slices (avc_conv_pack_slice modes 0-3: padded, flipped, per tap, padded Co)
    nm = Ci // 3 + 1
    slices = [(0, nm, nm + 7, 0), (0, nm, nm, 1), (nm, Ci - nm, Ci - nm, 2), (1, Ci - 2, Co + 5, 3)]
    ref = [Kr.conv_pack(w, 0, Kr.BF16), Kr.conv_pack(w, 1, Kr.BF16), Kr.convert(wih, Kr.BF16),
           Kr.transpose(whh, Kr.BF16), Kr.add(bih, bhh)]
    ref += [Kr.conv_pack_slice(w, *sl, Kr.BF16) for sl in slices]
    outs = [torch.empty_like(t) for t in ref]
    from autoformer_amd._lib import PACK_ADD, PACK_CONV_D, PACK_CONV_F, PACK_CONV_SLICE, PACK_COPY, PACK_TRANSPOSE
    ops = [{"src": w.data_ptr(), "dst": outs[0].data_ptr(), "kind": PACK_CONV_F, "dtype": Kr.BF16, "dims": (Co, Ci, 5)},
           {"src": w.data_ptr(), "dst": outs[1].data_ptr(), "kind": PACK_CONV_D, "dtype": Kr.BF16, "dims": (Co, Ci, 5)},
           {"src": wih.data_ptr(), "dst": outs[2].data_ptr(), "kind": PACK_COPY, "dtype": Kr.BF16, "dims": (G * In,)},
           {"src": whh.data_ptr(), "dst": outs[3].data_ptr(), "kind": PACK_TRANSPOSE, "dtype": Kr.BF16,
            "dims": (G, H), "ld": G},
           {"src": bih.data_ptr(), "src2": bhh.data_ptr(), "dst": outs[4].data_ptr(), "kind": PACK_ADD,
            "dtype": Kr.F32, "dims": (G,)}]
    ops += [{"src": w.data_ptr(), "dst": o.data_ptr(), "kind": PACK_CONV_SLICE, "dtype": Kr.BF16, "dims": (Co, Ci, 5),
             "slice": sl} for o, sl in zip(outs[5:], slices)]

    class _C:  # the PackCache surface _batch_plan reads
        pass
    c = _C()
    c.params, c.val, c.ops = [w, wih, whh, bih, bhh], tuple(outs), lambda val: ops
    plan = Lyr._batch_plan([c], group=99)
    Kr.L.call("avc_pack_batch", plan["ops"].data_ptr(), plan["prefix"].data_ptr(), plan["n"], plan["total"],
              Kr.stream())
    torch.cuda.synchronize()
    for a, b in zip(outs, ref):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B", [64, 20])
def test_lstm2_wavefront_forward(B):
    """Two stacked layers in one wavefront launch (decoder lstm2, AutoVC.py:96,110) against an
    fp32 CPU loop of the two layers with the kernel's roundings (h of both layers rounded to
    bf16 for the products, bf16 weights); the spin-timeout flag stays clear."""
    import autoformer_amd as A
    from autoformer_amd import kernels as Kr

    A.set_compute("bf16")
    H, T = 1024, 29
    G = 4 * H
    assert Kr.lstm2_persistent(B, H, H)
    torch.manual_seed(5)
    xproj = torch.randn(B * T, G) * 0.5
    ws = [(torch.randn(G, H) * (1.0 / H ** 0.5)).bfloat16() for _ in range(3)]
    bias1 = torch.randn(G) * 0.1
    h0, c0, g0, h1, c1, g1 = Kr.lstm2_fwd(xproj.to(DEV), *[w.to(DEV) for w in ws], bias1.to(DEV), B, T, H)
    torch.cuda.synchronize()
    assert int(Kr._CACHE["lstm2_buf"].view(torch.int32)[0].item()) == 0
    torch.testing.assert_close(h0._bf16.float(), h0.to(torch.bfloat16).float(), rtol=0, atol=0)
    w0, wi1, w1 = [w.float() for w in ws]
    xp = xproj.view(B, T, G)
    hs = [torch.zeros(B, H), torch.zeros(B, H)]
    cs = [torch.zeros(B, H), torch.zeros(B, H)]
    outs = [[], []]
    gts_out = [[], []]
    for t in range(T):
        for L in range(2):
            if L == 0:
                pre = xp[:, t] + hs[0].bfloat16().float() @ w0.t()
            else:
                pre = bias1 + outs[0][t].bfloat16().float() @ wi1.t() + hs[1].bfloat16().float() @ w1.t()
            i, f, gg, o = pre.chunk(4, 1)
            i, f, gg, o = torch.sigmoid(i), torch.sigmoid(f), torch.tanh(gg), torch.sigmoid(o)
            cs[L] = f * cs[L] + i * gg
            hs[L] = o * torch.tanh(cs[L])
            outs[L].append(hs[L])
            gts_out[L].append(torch.cat([i, f, gg, o], 1))
    for L, (h, c, g) in enumerate(((h0, c0, g0), (h1, c1, g1))):
        ref = torch.stack(outs[L], 1).reshape(B * T, H)
        assert relf(h, ref) < 3e-3, (L, relf(h, ref))
        assert relf(c.cpu().view(B, T, H)[:, -1], cs[L]) < 3e-3
        assert relf(g, torch.stack(gts_out[L], 1).reshape(B * T, G)) < 3e-3


def test_lstm2_wavefront_autograd_matches_layerwise():
    """layers.lstm over nn.LSTM(512, 1024, num_layers=2): the wavefront pair node gives the same
    output and parameter / input gradients as the layer-by-layer nodes (bf16 tolerance)."""
    import autoformer_amd as A
    from autoformer_amd import layers as Ly

    A.set_compute("bf16")
    Ly.set_grad_sink(False)
    B, T = 64, 24
    torch.manual_seed(6)
    mod = torch.nn.LSTM(512, 1024, num_layers=2, batch_first=True).to(DEV)
    cores = [Ly.LSTMLayerCore(mod, 0), Ly.LSTMLayerCore(mod, 1)]
    x0 = torch.randn(B * T, 512, device=DEV)
    res = []
    for off in (False, True):
        Ly._PAIR_OFF = off
        try:
            assert Ly._pair_ok(cores, x0, B) == (not off)
            mod.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_(True)
            y = Ly.lstm(mod, cores, x, B, T)
            (y * torch.linspace(-1, 1, 1024, device=DEV)).sum().backward()
            Ly.join_side()
            torch.cuda.synchronize()
            res.append((y.detach().clone(), x.grad.clone(), [p.grad.clone() for p in mod.parameters()]))
        finally:
            Ly._PAIR_OFF = False
    (ya, dxa, ga), (yb, dxb, gb) = res
    assert relf(ya, yb) < 1e-2, relf(ya, yb)
    assert relf(dxa, dxb) < 2e-2, relf(dxa, dxb)
    for a, b in zip(ga, gb):
        assert relf(a, b) < 2e-2, relf(a, b)


@pytest.mark.parametrize("out_bf16", [True, False])
@pytest.mark.parametrize("act_name", ["relu", "tanh"])
def test_gemm_bnb_matches_separate_bn_backward(out_bf16, act_name):
    """avc_gemm_bnb (the producing layer's BatchNorm backward statistics in the GEMM epilogue,
    last-row-tile finalize) + avc_bn_bwd_apply equal avc_bn_bwd's reduce / finalize / apply
    passes over the same GEMM output: dy, dgamma, dbeta and the conv-bias gradient."""
    import autoformer_amd as A
    from autoformer_amd import kernels as Kr

    A.set_compute("bf16")
    act = {"relu": Kr.ACT_RELU, "tanh": Kr.ACT_TANH}[act_name]
    M, N, Kd = 1000, 320, 256  # ragged row tiles (1000 = 7 x 128 + 104), 5 column tiles of 64
    torch.manual_seed(9)
    a = (torch.randn(M, Kd) * 0.5).bfloat16().to(DEV)
    w = (torch.randn(N, Kd) * 0.05).bfloat16().to(DEV)
    y = (torch.randn(M, N) * 1.3 + 0.2).bfloat16().to(DEV)
    mean = y.float().mean(0)
    rstd = 1.0 / (y.float().var(0, unbiased=False) + 1e-5).sqrt()
    gamma = (torch.rand(N) + 0.5).to(DEV)
    beta = (torch.randn(N) * 0.2).to(DEV)
    dt = torch.bfloat16 if out_bf16 else torch.float32
    c_ref = torch.empty(M, N, device=DEV, dtype=dt)
    Kr.gemm(M, N, Kd, Kr.operand(a, Kd), Kr.operand(w, Kd), c_ref)
    dy_ref, dg_ref, db_ref, dbi_ref = Kr.bn_bwd(c_ref, None, y, mean, rstd, gamma, act, beta=beta)
    c = torch.empty(M, N, device=DEV, dtype=dt)
    coef = torch.empty(6 * N, device=DEV)
    dg, db, dbi = (torch.full((N,), 0.25, device=DEV) for _ in range(3))  # accumulate onto 0.25
    Kr.gemm(M, N, Kd, Kr.operand(a, Kd), Kr.operand(w, Kd), c,
            bnb=(y, mean, rstd, gamma, beta, act, coef, dg, db, dbi, 1))
    dy = Kr.bn_bwd_apply(c, y, coef, act)
    torch.cuda.synchronize()
    torch.testing.assert_close(c, c_ref, rtol=0, atol=0)
    assert relf(dy, dy_ref) < 1e-5, relf(dy, dy_ref)
    assert relf(dg - 0.25, dg_ref) < 1e-5
    assert relf(db - 0.25, db_ref) < 1e-5
    # the conv-bias gradient of a conv feeding training-mode BN is analytically zero: both sides
    # are cancellation residue of sums whose terms have dbeta's scale (plus 0.25's fp32 ulp)
    tol = 1e-5 * float(db_ref.abs().max()) + 4 * 2.0 ** -25
    assert float((dbi - 0.25 - dbi_ref).abs().max()) < tol, float((dbi - 0.25 - dbi_ref).abs().max())


@pytest.mark.parametrize("T", [64, 128])
def test_conv_chain_fused_bn_backward_matches_separate(T):
    """Three conv_bn layers (the encoder chain, AutoVC.py:46-58) with fuse_prev: output and every
    parameter / input gradient equal the chain run with the fusion off (AVC_BNB=0 path).  T = 128:
    the data-gradient convs run on the halo conv ring with its BN-backward epilogue
    (ring_bnb_epilogue); T = 64: the links are not made (the ring does not take those convs), both
    runs take the separate passes."""
    import autoformer_amd as A
    from autoformer_amd import layers as Ly
    from autoformer_amd import kernels as Kr

    A.set_compute("bf16")
    Ly.set_grad_sink(False)
    B, C = 8, 512
    torch.manual_seed(10)
    mods = []
    for i in range(3):
        conv = torch.nn.Conv1d(C if i else 80, C, 5, padding=2).to(DEV)
        bn = torch.nn.BatchNorm1d(C).to(DEV).train()
        with torch.no_grad():
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.normal_(0, 0.1)
        mods += [conv, bn]
    cores = [Ly.ConvBNCore(mods[2 * i], mods[2 * i + 1], Kr.ACT_RELU) for i in range(3)]
    x0 = torch.randn(B * T, 80, device=DEV)
    res = []
    saved = Ly._BNB_ON
    for on in (True, False):
        Ly._BNB_ON = on
        try:
            for m in mods:
                m.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_(True)
            h = Ly.conv_bn(cores[0], x, B, T, out_bf16=True)
            h = Ly.conv_bn(cores[1], h, B, T, out_bf16=True, fuse_prev=True)
            h = Ly.conv_bn(cores[2], h, B, T, fuse_prev=True)
            (h.float() * torch.linspace(-1, 1, C, device=DEV)).sum().backward()
            torch.cuda.synchronize()
            res.append((h.detach().float().clone(), x.grad.clone(),
                        [p.grad.clone() for m in mods for p in m.parameters()]))
        finally:
            Ly._BNB_ON = saved
    (ha, dxa, ga), (hb, dxb, gb) = res
    torch.testing.assert_close(ha, hb, rtol=0, atol=0)
    assert relf(dxa, dxb) < 2e-3, relf(dxa, dxb)
    for p, q in zip(ga, gb):
        assert relf(p, q) < 2e-3 or float((p - q).abs().max()) < 1e-4, relf(p, q)


@pytest.mark.parametrize("n1,n2,off", [(64 * 128 * 80, 64 * 8 * 88, 0), (1001, 37, 1), (5, 0, 0)])
def test_vc_loss_block_matches_torch(n1, n2, off):
    """avc_vc_loss / avc_vc_loss_grad (the fused loss block of train.py:84-96) against
    F.mse_loss / F.l1_loss in fp64: values, the weighted total, and the gradients for upstream
    gradients on the total AND on the separate terms (off = 1: unaligned, scalar-load path)."""
    from autoformer_amd.train import vc_loss_block

    torch.manual_seed(3)
    x = torch.randn(n1).to(DEV)
    y1 = (torch.randn(n1) * 0.7).to(DEV)
    y2 = (torch.randn(n1) * 1.3).to(DEV)
    if off:  # misaligned views into a larger buffer
        big = torch.randn(3 * n1 + 3, device=DEV)
        x, y1, y2 = big[1:1 + n1], big[n1 + 2:2 * n1 + 2], big[2 * n1 + 3:3 * n1 + 3]
    ca, cb = torch.randn(max(n2, 1)).to(DEV)[:n2], torch.randn(max(n2, 1)).to(DEV)[:n2]
    lam = 0.75
    y1r, y2r, car, cbr = (t.detach().clone().requires_grad_(True) for t in (y1, y2, ca, cb))
    total, (l_id, l_ps, l_cd) = vc_loss_block(x, y1r, y2r, car, cbr, lam)
    xd, y1d, y2d, cad, cbd = (t.detach().cpu().double().requires_grad_(True) for t in (x, y1, y2, ca, cb))
    r_id = F.mse_loss(y1d, xd)
    r_ps = F.mse_loss(y2d, xd)
    r_cd = F.l1_loss(cad, cbd) if n2 else torch.zeros((), dtype=torch.float64)
    r_tot = r_id + r_ps + lam * r_cd
    for a, b in ((l_id, r_id), (l_ps, r_ps), (l_cd, r_cd), (total, r_tot)):
        assert abs(float(a) - float(b)) <= 1e-5 * max(abs(float(b)), 1e-6), (float(a), float(b))
    (2.0 * total + 0.5 * l_ps + 3.0 * l_cd).backward()
    (2.0 * r_tot + 0.5 * r_ps + 3.0 * r_cd).backward()
    assert relf(y1r.grad, y1d.grad) < 1e-5
    assert relf(y2r.grad, y2d.grad) < 1e-5
    if n2:
        assert relf(car.grad, cad.grad) < 1e-5
        assert relf(cbr.grad, cbd.grad) < 1e-5


@pytest.mark.parametrize("ydt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,C", [(1001, 520), (8192, 512), (37, 80), (50, 84)])
def test_bn_apply_forms(ydt, M, C):
    """avc_bn_apply / avc_bn_bwd_apply (8-channel row-looping forms when C % 8 == 0, 4-channel /
    scalar otherwise; ragged row counts) against torch fp32 of the same formulas."""
    from autoformer_amd import kernels as Kr

    torch.manual_seed(5)
    y = (torch.randn(M, C) * 2 + 0.3).to(ydt).to(DEV)
    yf = y.float()
    scale, shift = (torch.rand(C) + 0.5).to(DEV), torch.randn(C).to(DEV)
    res = torch.randn(M, C, device=DEV)
    for act, fn in ((Kr.ACT_RELU, torch.relu), (Kr.ACT_TANH, torch.tanh)):
        ref = fn(yf * scale + shift)
        out = Kr.bn_apply(y, scale, shift, act)
        assert relf(out, ref) < 1e-6
        out = Kr.bn_apply(y, scale, shift, act, residual=res)
        assert relf(out, ref + res) < 1e-6
        o16 = Kr.bn_apply(y, scale, shift, act, out_bf16=True)
        assert o16.dtype == torch.bfloat16 and relf(o16, ref) < 4e-3
    k1, m1, m2, mu, rs, bt = (torch.rand(C) + 0.5, torch.randn(C) * 0.1, torch.randn(C) * 0.1, torch.randn(C) * 0.2,
                              torch.rand(C) + 0.5, torch.randn(C) * 0.3)
    coef = torch.cat([k1, m1, m2, mu, rs, bt]).to(DEV)
    k1, m1, m2, mu, rs, bt = (t.to(DEV) for t in (k1, m1, m2, mu, rs, bt))
    dA = torch.randn(M, C).to(ydt).to(DEV)
    for act in (Kr.ACT_RELU, Kr.ACT_TANH):
        yc = yf - mu
        z = yc * k1 + bt
        der = (z > 0).float() if act == Kr.ACT_RELU else 1 - torch.tanh(z) ** 2
        ref = k1 * (dA.float() * der - m1 - yc * rs * m2)
        dy = Kr.bn_bwd_apply(dA, y, coef, act)
        assert relf(dy, ref) < 1e-5, relf(dy, ref)
        d16 = Kr.bn_bwd_apply(dA, y, coef, act, dy_bf16=True)
        assert d16.dtype == torch.bfloat16 and relf(d16, ref) < 4e-3


# ------------------------------------------------------------------ encoder conv0 fold (fold.hip)
@pytest.mark.parametrize("comp", ["fp32", "bf16"])
def test_fold_kernels(comp):
    """avc_conv_pack_slice (3 modes), avc_conv_edge_table, avc_conv_edge_colsum (fp32 / bf16 dy),
    avc_conv_grad_unpack_slice and the GEMM row-bias epilogue against torch restatements."""
    import autoformer_amd as A
    from autoformer_amd import kernels as Kr
    from tests.capture_ref import row_bias_rows

    A.set_compute(comp)
    dt = Kr.compute()
    tdt = torch.bfloat16 if comp == "bf16" else torch.float32
    torch.manual_seed(3)
    Co, Ci, Kw, nm, cp = 48, 40, 5, 10, 32
    w = torch.randn(Co, Ci, Kw, device=DEV)
    f = Kr.conv_pack_slice(w, 0, nm, cp, 0, dt)
    ref = torch.zeros(Co, Kw, cp, device=DEV)
    ref[:, :, :nm] = w[:, :nm].permute(0, 2, 1)
    assert torch.equal(f.float(), ref.reshape(Co, Kw * cp).to(tdt).float())
    d = Kr.conv_pack_slice(w, 0, nm, nm, 1, dt)
    refd = w[:, :nm].flip(2).permute(1, 2, 0).reshape(nm, Kw * Co)
    assert torch.equal(d.float(), refd.to(tdt).float())
    e = Kr.conv_pack_slice(w, nm, Ci - nm, Ci - nm, 2, dt)
    refe = w[:, nm:].permute(2, 0, 1).reshape(Kw * Co, Ci - nm)
    assert torch.equal(e.float(), refe.to(tdt).float())
    B, T, pad = 3, 13, 2
    E = torch.randn(B, Kw * Co, device=DEV)
    S = Kr.conv_edge_table(E, B, Co, Kw, T, pad)
    Ev = E.view(B, Kw, Co)
    for cls, t in enumerate([0, 1, 2, T - 2, T - 1]):
        want = sum(Ev[:, k] for k in range(Kw) if 0 <= t + k - pad < T)
        assert (S.view(B, 5, Co)[:, cls] - want).abs().max() < 1e-5
    dy = torch.randn(B * T, Co, device=DEV).to(tdt)
    Sdy = Kr.conv_edge_colsum(dy, B, T, Co, Kw, pad).view(B, Kw, Co)
    dv = dy.float().view(B, T, Co)
    for k in range(Kw):
        assert (Sdy[:, k] - dv[:, max(0, pad - k):min(T, T + pad - k)].sum(1)).abs().max() < 1e-3
    g = torch.randn(Co, Ci, Kw, device=DEV)
    g0 = g.clone()
    dwf = torch.randn(Co, Kw * 16, device=DEV)
    Kr.conv_grad_unpack_slice(dwf, Kw * 16, 16, g, 12, 9)
    want = g0.clone()
    want[:, 12:21] += dwf.view(Co, Kw, 16)[:, :, :9].permute(0, 2, 1)
    assert (g - want).abs().max() < 1e-6
    # row bias on a 5-tap window GEMM (the conv kernel in bf16 mode: 32-multiple channels)
    C2, N2 = 64, 96
    x = torch.randn(B * T, C2, device=DEV).to(tdt)
    W2 = (torch.randn(N2, Kw * C2, device=DEV) * 0.1).to(tdt)
    S2 = torch.randn(B * 5, N2, device=DEV)
    y = torch.empty(B * T, N2, device=DEV)
    Kr.gemm(B * T, N2, Kw * C2, Kr.operand(x, C2, window=(Kw, pad, T, T, C2)), Kr.operand(W2, Kw * C2), y,
            row_bias=(S2, T, pad))
    xs = torch.nn.functional.pad(x.double().view(B, T, C2), (0, 0, pad, pad))
    im = torch.cat([xs[:, k:k + T] for k in range(Kw)], 2).reshape(B * T, Kw * C2)
    refy = im @ W2.double().t() + row_bias_rows(S2, B * T, T, pad)
    assert relf(y, refy) < 1e-5, relf(y, refy)


@pytest.mark.parametrize("comp", ["fp32", "bf16"])
def test_enc_conv0_fold_matches_concat(comp):
    """The folded encoder conv0 (layers._EncConv0FoldFn) against the concat form
    (_EncConv0Fn) on the same weights and inputs: activation, BN running statistics, dL/dmel,
    dL/demb and every parameter gradient (fp32: 1e-5; bf16: the bf16 bar of the layer)."""
    import autoformer_amd as A
    from autoformer_amd import layers as Lyr
    from autoformer_amd.factory.Norm import ConvNorm

    A.set_compute(comp)
    torch.manual_seed(4)
    B, T, nm, de, Co = 4, 32, 80, 256, 512
    res = []
    for fold in (True, False):
        torch.manual_seed(4)
        conv = ConvNorm(nm + de, Co, kernel_size=5, stride=1, padding=2, dilation=1, w_init_gain="relu").conv.to(DEV)
        bn = torch.nn.BatchNorm1d(Co).to(DEV)
        core = Lyr.ConvBNCore(conv, bn, Kr_act_relu())
        mel = torch.randn(B * T, nm, device=DEV, requires_grad=True)
        emb = torch.nn.functional.normalize(torch.randn(B, de, device=DEV), dim=1).requires_grad_(True)
        fn = Lyr._EncConv0FoldFn if fold else Lyr._EncConv0Fn
        a = fn.apply(mel, emb, core, B, T, False, conv.weight, conv.bias, bn.weight, bn.bias)
        (a.float() * torch.linspace(-1, 1, Co, device=DEV)).sum().backward()
        torch.cuda.synchronize()
        res.append((a.float(), mel.grad, emb.grad, conv.weight.grad, bn.weight.grad, bn.bias.grad, bn.running_mean,
                    bn.running_var))
    # bf16: two bf16 computations of the same layer whose fp32 sums run in different orders; the
    # ReLU after BN flips units with a near-zero pre-activation, which moves dL/dmel by ~3 %
    bar = 1e-5 if comp == "fp32" else 5e-2
    names = ("a", "dmel", "demb", "dW", "dgamma", "dbeta", "running_mean", "running_var")
    for n, u, v in zip(names, res[0], res[1]):
        assert relf(u, v.double()) < bar, (n, relf(u, v.double()))


def Kr_act_relu():
    from autoformer_amd import kernels as Kr
    return Kr.ACT_RELU


@pytest.mark.parametrize("B,T,Cin,Cout", [(64, 128, 512, 512), (3, 37, 64, 96), (5, 50, 96, 136), (8, 176, 512, 80),
                                          (2, 300, 32, 64)])
def test_conv_bn_fused_finalize(B, T, Cin, Cout):
    """The halo conv kernels with the BN finalize in their epilogue (the forward conv + BN of every
    ConvNorm layer) against the same conv with the separate finalize: y, partials, mean / rstd /
    scale / shift and the running statistics.  Utterance-aligned shapes (T % 128 == 0) take the
    eight-wave ring kernel (gemm_ring.hip conv_ring_kernel), the others gemm_conv.hip."""
    import autoformer_amd as A
    from autoformer_amd import kernels as Kr

    A.set_compute("bf16")
    torch.manual_seed(11)
    M = B * T
    x = torch.randn(M, Cin, device=DEV).bfloat16()
    Wf = (torch.randn(Cout, 5 * Cin, device=DEV) * 0.1).bfloat16()
    bias = torch.randn(Cout, device=DEV)
    gamma, beta = (torch.rand(Cout) + 0.5).to(DEV), torch.randn(Cout).to(DEV)
    rm0, rv0 = torch.randn(Cout).to(DEV), (torch.rand(Cout) + 0.5).to(DEV)
    outs = []
    for fused in (True, False):
        y = torch.empty(M, Cout, device=DEV)
        p = Kr.bn_partial_buffer(M, Cout, DEV)
        rm, rv, n = rm0.clone(), rv0.clone(), torch.zeros((), dtype=torch.long, device=DEV)
        xo, wo = Kr.operand(x, Cin, window=(5, 2, T, T, Cin)), Kr.operand(Wf, 5 * Cin)
        if fused:
            st = Kr.gemm(M, Cout, 5 * Cin, xo, wo, y, bias=bias, bn_partial=p,
                         bn_fin=(gamma, beta, rm, rv, n, 0.1, 1e-5, 1))
        else:
            Kr.gemm(M, Cout, 5 * Cin, xo, wo, y, bias=bias, bn_partial=p)
            st = Kr.bn_finalize(p, M, Cout, gamma, beta, rm, rv, n, 0.1, 1e-5)
        torch.cuda.synchronize()
        outs.append((y, p, st, rm, rv))
    (y1, p1, s1, rm1, rv1), (y2, p2, s2, rm2, rv2) = outs
    assert torch.equal(y1, y2) and torch.equal(p1, p2)
    for a, b in zip(s1, s2):
        assert rinf(a, b) < 1e-6
    assert rinf(rm1, rm2) < 1e-6 and rinf(rv1, rv2) < 1e-6
    yf = y1.double()
    assert rinf(s1[0], yf.mean(0)) < 1e-5
    assert rinf(s1[1], 1 / torch.sqrt(yf.var(0, unbiased=False) + 1e-5)) < 1e-4


# ------------------------------------------------------------------ Discriminator head (disc.hip)
@pytest.mark.parametrize("B,nl,nc", [(64, 74, 22), (5, 9, 7), (300, 3, 130)])
def test_disc_dense_head(B, nl, nc):
    """sigmoid(dense1(flatten(a))) with the channel-major flatten of Discriminator.py:28-29 on a
    bin-major activation, and its backward from dL/dp, against fp64 autograd."""
    from autoformer_amd import kernels as K

    a = torch.randn(B, nl, nc)
    w = torch.randn(1, nc * nl) * 0.1
    bias = torch.randn(1)
    dp = torch.randn(B, 1)
    a64, w64, b64 = (t.double().requires_grad_() for t in (a, w, bias))
    # reference flatten: (B, C, L) channel-major
    p64 = torch.sigmoid(a64.transpose(1, 2).reshape(B, nc * nl) @ w64.t() + b64)
    p64.backward(dp.double())
    ad, wd, bd = a.to(DEV).reshape(B, nl * nc), w.to(DEV), bias.to(DEV)
    p = K.disc_dense_fwd(ad, wd, bd, B, nl, nc)
    da, dw, db = K.disc_dense_bwd(dp.to(DEV), p, ad, wd, B, nl, nc)
    assert rinf(p, p64.detach()) < 1e-5
    assert relf(da.view(B, nl, nc), a64.grad) < 1e-5
    assert relf(dw, w64.grad) < 1e-5
    assert relf(db, b64.grad) < 1e-5


def test_conv_pack_slice_output_padded():
    """conv_pack_slice mode 3 (data-gradient pack with the output-channel axis zero-padded):
    Wd[ci][k'][co] = w[co][ci][K-1-k'] for co < Co, 0 in the pad -- conv_pack mode 1 widened."""
    from autoformer_amd import kernels as Kr

    w = torch.randn(22, 44, 3)
    got = Kr.conv_pack_slice(w.to(DEV), 0, 44, 24, 3, Kr.F32).cpu().view(44, 3, 24)
    ref = torch.zeros(44, 3, 24)
    ref[:, :, :22] = w.flip(2).permute(1, 2, 0)
    assert torch.equal(got, ref)
    base = Kr.conv_pack(w.to(DEV), 1, Kr.F32).cpu().view(44, 3, 22)
    assert torch.equal(got[:, :, :22], base)
