"""The deep-ring GEMM kernels (gemm_ring.hip) against fp32 references of the same op:

  * gemm_ring_kernel at every tile configuration, with ragged M / N / K (zero-granule tails), bias,
    residual, accumulate, bf16 twin and the batch fold of shared-B products
    (reference: the nn.Linear / Conv1d(k=1) products of factory/MLPMixer.py:16-33,58-92);
  * conv_ring_kernel (5-tap 'same' Conv1d, factory/Norm.py:21-28) on utterance-aligned and
    straddling tiles, with the BatchNorm statistics + finalize epilogue;
  * the fused GELU epilogues (avc_gemm_desc.c_bf16_act / act_grad_of, MLPMixer.py:9-23) and the
    bias-gradient column sums (col_sum), on the ring kernel and on the fallback pass after the
    older kernels.
Operands are bf16 (exact in fp32), so the references are fp32 products of the same values.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _ring(mode, bm=0, bn=0, nst=0, gm=8, win=2):
    from autoformer_amd import _lib

    _lib.call("avc_gemm_set_ring", mode, bm, bn, nst, gm, win)


@pytest.fixture(autouse=True)
def _bf16_and_reset():
    import autoformer_amd as A

    A.set_compute("bf16")
    yield
    _ring(-1)


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


CFGS = [(256, 256, 2), (256, 128, 3), (128, 128, 4), (128, 128, 3), (128, 256, 3), (256, 128, 2),
        (256, 256, 14), (256, 128, 15), (128, 128, 16), (128, 128, 2)]  # nst 10 + n: 32-deep slots (gemm_ring32_kernel)


@pytest.mark.parametrize("cfg", CFGS)
@pytest.mark.parametrize("M,N,Kd", [(1000, 300, 200), (513, 1100, 72), (256, 256, 64)])
def test_ring_gemm_configs(cfg, M, N, Kd):
    from autoformer_amd import kernels as K

    torch.manual_seed(M + N + Kd)
    a = torch.randn(M, Kd, device=DEV).bfloat16()
    b = torch.randn(N, Kd, device=DEV).bfloat16()
    bias = torch.randn(N, device=DEV)
    res = torch.randn(M, N, device=DEV)
    ref = a.float() @ b.float().t() + bias + res
    _ring(1, *cfg)
    c = torch.empty(M, N, device=DEV)
    c16 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    K.gemm(M, N, Kd, K.operand(a, Kd), K.operand(b, Kd), c, bias=bias, residual=res, c_bf16=c16)
    torch.cuda.synchronize()
    assert _rel(c, ref) < 1e-5
    assert _rel(c16.float(), ref) < 1e-2
    # bf16-only output (the 16-B bf16 store path of the ring epilogue), no residual
    o16 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    K.gemm(M, N, Kd, K.operand(a, Kd), K.operand(b, Kd), o16, bias=bias)
    torch.cuda.synchronize()
    assert _rel(o16.float(), ref - res) < 1e-2
    # accumulate on top
    c2 = c.clone()
    K.gemm(M, N, Kd, K.operand(a, Kd), K.operand(b, Kd), c2, accumulate=True)
    torch.cuda.synchronize()
    assert _rel(c2, c + a.float() @ b.float().t()) < 1e-5


def test_ring_default_policy_and_batch_fold():
    """The MetaConv token-mixing shape at reduced batch: a batch of per-utterance products sharing B
    is folded into one product (344-row utterances, no per-batch row-tile remainder)."""
    from autoformer_amd import kernels as K

    torch.manual_seed(3)
    B, D, NPp, N4 = 6, 344, 1856, 4 * 1856
    a = torch.randn(B * D, NPp, device=DEV).bfloat16()
    w = (torch.randn(N4, NPp, device=DEV) * 0.05).bfloat16()
    bias = torch.randn(N4, device=DEV)
    c = torch.empty(B * D, N4, device=DEV)
    K.gemm(D, N4, NPp, K.operand(a, NPp, batch_stride=D * NPp), K.operand(w, NPp), c, bias=bias, batch=B,
           c_batch_stride=D * N4)
    torch.cuda.synchronize()
    assert _rel(c, a.float() @ w.float().t() + bias) < 1e-5


@pytest.mark.parametrize("B,T,Cin,Cout,forced", [(8, 128, 512, 512, False), (4, 256, 64, 136, False),
                                                  (3, 176, 96, 200, True), (2, 50, 32, 64, True)])
@pytest.mark.parametrize("bn", [False, True])
def test_conv_ring(B, T, Cin, Cout, forced, bn):
    from autoformer_amd import kernels as K

    torch.manual_seed(B * T + Cin)
    M = B * T
    x = torch.randn(M, Cin, device=DEV).bfloat16()
    Wf = (torch.randn(Cout, 5 * Cin, device=DEV) * 0.1).bfloat16()
    bias = torch.randn(Cout, device=DEV)
    xp = torch.nn.functional.pad(x.float().view(B, T, Cin), (0, 0, 2, 2))
    win = torch.cat([xp[:, k:k + T] for k in range(5)], dim=2).reshape(M, 5 * Cin)
    ref = win @ Wf.float().t() + bias
    outs = []
    # ring (forced for straddling tiles), old
    ring = (1, 128, 128, 4) if forced else (-1,)
    for mode in (ring, (0,)):
        _ring(*mode)
        y = torch.empty(M, Cout, device=DEV)
        xo, wo = K.operand(x, Cin, window=(5, 2, T, T, Cin)), K.operand(Wf, 5 * Cin)
        if bn:
            p = K.bn_partial_buffer(M, Cout, DEV)
            g_, b_ = torch.ones(Cout, device=DEV), torch.zeros(Cout, device=DEV)
            rm, rv = torch.zeros(Cout, device=DEV), torch.ones(Cout, device=DEV)
            st = K.gemm(M, Cout, 5 * Cin, xo, wo, y, bias=bias, bn_partial=p, bn_fin=(g_, b_, rm, rv, None, 0.1, 1e-5, 1))
        else:
            st = None
            K.gemm(M, Cout, 5 * Cin, xo, wo, y, bias=bias)
        torch.cuda.synchronize()
        outs.append((y, st))
        assert _rel(y, ref) < 1e-5, mode
        if bn:
            assert _rel(st[0], ref.mean(0)) < 1e-5
            assert _rel(st[1], 1 / torch.sqrt(ref.var(0, unbiased=False) + 1e-5)) < 1e-4


@pytest.mark.parametrize("B,T,Cin,Cout", [(4, 176, 64, 200), (64, 176, 512, 512), (3, 160, 96, 136), (2, 192, 32, 128)])
@pytest.mark.parametrize("bn", [False, True])
def test_conv_utterance_tile(B, T, Cin, Cout, bn):
    """conv_utt_kernel: one utterance per 192-row tile (128 < T <= 192; T = 176 is C4 / C5), rows
    T..191 computed from zero halo rows and not stored; the BatchNorm statistics as one T-row tile
    per workgroup, merged by the in-kernel finalize (bn_rows = T)."""
    from autoformer_amd import _lib
    from autoformer_amd import kernels as K

    torch.manual_seed(B * T + Cin + Cout)
    M = B * T
    x = torch.randn(M, Cin, device=DEV).bfloat16()
    Wf = (torch.randn(Cout, 5 * Cin, device=DEV) * 0.1).bfloat16()
    bias = torch.randn(Cout, device=DEV)
    xp = torch.nn.functional.pad(x.float().view(B, T, Cin), (0, 0, 2, 2))
    win = torch.cat([xp[:, k:k + T] for k in range(5)], dim=2).reshape(M, 5 * Cin)
    ref = win @ Wf.float().t() + bias
    _ring(-1)
    y = torch.full((M + 64, Cout), 7.0, device=DEV)  # rows past M must stay untouched
    xo, wo = K.operand(x, Cin, window=(5, 2, T, T, Cin)), K.operand(Wf, 5 * Cin)
    if bn:
        p = K.bn_partial_buffer(M, Cout, DEV)
        g_, b_ = torch.rand(Cout, device=DEV) + 0.5, torch.randn(Cout, device=DEV)
        rm, rv = torch.zeros(Cout, device=DEV), torch.ones(Cout, device=DEV)
        nbt = torch.zeros(1, device=DEV, dtype=torch.int64)
        st = K.gemm(M, Cout, 5 * Cin, xo, wo, y, bias=bias, bn_partial=p, bn_fin=(g_, b_, rm, rv, nbt, 0.1, 1e-5, 1))
    else:
        K.gemm(M, Cout, 5 * Cin, xo, wo, y, bias=bias)
    assert _lib.lib().avc_gemm_ring_last() == 3, "the one-utterance halo conv did not run"
    y16 = torch.empty(M, Cout, device=DEV, dtype=torch.bfloat16)
    K.gemm(M, Cout, 5 * Cin, xo, wo, y16, bias=bias)  # bf16-only output (the 16-B store path)
    torch.cuda.synchronize()
    assert _rel(y[:M], ref) < 1e-5
    assert bool((y[M:] == 7.0).all())
    assert _rel(y16.float(), ref) < 1e-2
    if bn:
        mean, var = ref.double().mean(0), ref.double().var(0, unbiased=False)
        assert _rel(st[0], mean) < 1e-5
        assert _rel(st[1], 1 / torch.sqrt(var + 1e-5)) < 1e-4
        assert _rel(st[2], g_.double() / torch.sqrt(var + 1e-5)) < 1e-4
        assert _rel(rm, 0.1 * mean) < 1e-5
        assert _rel(rv, 0.9 + 0.1 * ref.double().var(0, unbiased=True)) < 1e-5
        assert int(nbt.item()) == 1


def _gelu_grad(x):
    xd = x.double()
    return 0.5 * (1 + torch.erf(xd / 2 ** 0.5)) + xd * torch.exp(-0.5 * xd * xd) / (2 * torch.pi) ** 0.5


@pytest.mark.parametrize("ring", [-1, 0])
@pytest.mark.parametrize("store", ["f32", "bf16"])
def test_gelu_epilogues(ring, store):
    """c_bf16_act = GELU and act_grad_of on the ring kernel (-1: N >= 1024) and on the pass after
    the older kernels (0); store = bf16: the pre-activation goes out in bf16 only (c_pre_bf16), the
    backward reads it (act_grad_dtype bf16) and writes its gradient in bf16 only."""
    from autoformer_amd import kernels as K

    torch.manual_seed(5)
    M, N, Kd = 1024, 1376, 344
    a = torch.randn(M, Kd, device=DEV).bfloat16()
    b = (torch.randn(N, Kd, device=DEV) * 0.1).bfloat16()
    bias = torch.randn(N, device=DEV)
    x = torch.randn(M, N, device=DEV)
    if store == "bf16":
        x = x.bfloat16()
    dt = torch.float32 if store == "f32" else torch.bfloat16
    _ring(ring)
    u = torch.empty(M, N, device=DEV, dtype=dt)
    v = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    K.gemm(M, N, Kd, K.operand(a, Kd), K.operand(b, Kd), u, bias=bias, c_bf16=v, c_bf16_act=K.ACT_GELU)
    d = torch.empty(M, N, device=DEV, dtype=dt)
    d16 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16) if store == "f32" else None
    K.gemm(M, N, Kd, K.operand(a, Kd), K.operand(b, Kd), d, c_bf16=d16, act_grad_of=x)
    torch.cuda.synchronize()
    uref = a.float() @ b.float().t() + bias
    dref = (a.float() @ b.float().t()).double() * _gelu_grad(x)
    tol = 1e-5 if store == "f32" else 5e-3  # bf16 stores: 2^-9 relative rounding
    assert _rel(u.float(), uref) < tol
    assert _rel(v.float(), torch.nn.functional.gelu(uref.double())) < 1e-2
    assert _rel(d.float(), dref) < tol
    if d16 is not None:
        assert _rel(d16.float(), dref) < 1e-2


@pytest.mark.parametrize("ring", [-1, 0])
@pytest.mark.parametrize("batch", [1, 3, 12])
@pytest.mark.parametrize("store", ["f32", "bf16"])
def test_col_sum_epilogue(ring, batch, store):
    """col_sum[:n] += column sums of the stored (GELU-backward) values, over every row of every
    folded batch, with a padded leading dimension (n < N: the token mixer's 4*NP of 4*NPp); with
    a bf16-only store the sums are of the fp32 values (ring) or of the stored bf16 (fallback).
    batch 12 (4128 rows) takes the slotted form (32 row-tile slots + a reduce pass that leaves the
    slots zeroed): the product runs twice and the second call must add the same sums again."""
    from autoformer_amd import kernels as K

    torch.manual_seed(7 + batch)
    M, N, Kd, n = 344, 1408, 192, 1300
    a = torch.randn(batch * M, Kd, device=DEV).bfloat16()
    b = (torch.randn(N, Kd, device=DEV) * 0.1).bfloat16()
    x = torch.randn(batch * M, N, device=DEV)
    if store == "bf16":
        x = x.bfloat16()
    _ring(ring)
    if store == "f32":
        d = torch.empty(batch * M, N, device=DEV)
        d16 = torch.empty(batch * M, N, device=DEV, dtype=torch.bfloat16)
    else:
        d, d16 = torch.empty(batch * M, N, device=DEV, dtype=torch.bfloat16), None
    cs = torch.randn(n + 5, device=DEV)
    cs0 = cs.clone()
    K.gemm(M, N, Kd, K.operand(a, Kd, batch_stride=M * Kd), K.operand(b, Kd), d, c_bf16=d16, act_grad_of=x,
           batch=batch, c_batch_stride=M * N, col_sum=cs, col_sum_n=n)
    torch.cuda.synchronize()
    dref = (a.float() @ b.float().t()).double() * _gelu_grad(x)
    tol = 1e-5 if store == "f32" else 5e-3
    assert _rel(d.float(), dref) < tol
    assert _rel(cs[:n] - cs0[:n], dref[:, :n].sum(0)) < tol
    assert torch.equal(cs[n:], cs0[n:])
    cs1 = cs.clone()
    K.gemm(M, N, Kd, K.operand(a, Kd, batch_stride=M * Kd), K.operand(b, Kd), d, c_bf16=d16, act_grad_of=x,
           batch=batch, c_batch_stride=M * N, col_sum=cs, col_sum_n=n)
    torch.cuda.synchronize()
    assert _rel(cs[:n] - cs1[:n], dref[:, :n].sum(0)) < tol
    assert torch.equal(cs[n:], cs0[n:])


@pytest.mark.parametrize("ring", [-1, 0])
@pytest.mark.parametrize("B,D,NP,Kd", [(5, 344, 1849, 512), (3, 176, 121, 512), (2, 8, 37, 64)])
def test_transposed_store(ring, B, D, NP, Kd):
    """c_trans_rows = D: the per-utterance (D x NP) products Z1_b = Z_b + (V_b W^T + b)^T written
    straight into the frame-major (NP x D) layout with the residual read there (the MLP-Mixer
    token FF output, MLPMixer.py:80-86), on the ring kernel and on the older kernels' epilogue."""
    from autoformer_amd import kernels as K

    torch.manual_seed(B + D)
    v = torch.randn(B * D, Kd, device=DEV).bfloat16()
    w = (torch.randn(NP, Kd, device=DEV) * 0.1).bfloat16()
    bias = torch.randn(NP, device=DEV)
    z = torch.randn(B * NP, D, device=DEV)
    _ring(ring)
    z1 = torch.empty(B * NP, D, device=DEV)
    K.gemm(D, NP, Kd, K.operand(v, Kd, batch_stride=D * Kd), K.operand(w, Kd), z1, bias=bias, batch=B,
           c_batch_stride=D * NP, residual=z, c_trans_rows=D)
    torch.cuda.synchronize()
    rt = (v.float() @ w.float().t() + bias).view(B, D, NP)
    ref = z + rt.transpose(1, 2).reshape(B * NP, D)
    assert _rel(z1, ref) < 1e-5


def test_generic_gemm_fused_gelu_outputs():
    """A non-vectorisable operand (odd row stride) sends the fused-GELU products to the generic kernel
    (fp32 C only) + the GELU pass: with an fp32 C both bf16 outputs are made from it --
    GELU(C) and, when asked for, the bf16 pre-activation slot (c_pre_bf16); a bf16-only output has
    no fp32 C to make them from and must be refused with an error, not a fault."""
    from autoformer_amd import _lib
    from autoformer_amd import kernels as K

    torch.manual_seed(11)
    M, N, Kd = 256, 320, 96
    abuf = torch.randn(M, Kd + 1, device=DEV).bfloat16()  # ld = 97: rows not 16-B aligned
    b = (torch.randn(N, Kd, device=DEV) * 0.1).bfloat16()
    u = torch.empty(M, N, device=DEV)
    v = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    K.gemm(M, N, Kd, K.operand(abuf, Kd + 1), K.operand(b, Kd), u, c_bf16=v, c_bf16_act=K.ACT_GELU)
    torch.cuda.synchronize()
    ref = abuf[:, :Kd].float() @ b.float().t()
    assert _rel(u, ref) < 1e-5
    assert _rel(v.float(), torch.nn.functional.gelu(ref.double())) < 1e-2
    # the bf16 pre-activation form: pre-activation and activation in bf16 only, no fp32 C
    pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="bf16-only output"):
        K.gemm(M, N, Kd, K.operand(abuf, Kd + 1), K.operand(b, Kd), pre, c_bf16=v, c_bf16_act=K.ACT_GELU)
    # a bf16-only GELU-backward output
    x = torch.randn(M, N, device=DEV)
    d = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="bf16-only output"):
        K.gemm(M, N, Kd, K.operand(abuf, Kd + 1), K.operand(b, Kd), d, act_grad_of=x)
    torch.cuda.synchronize()
    assert _lib.lib().avc_abi_version() == _lib.ABI_VERSION
