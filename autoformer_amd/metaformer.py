"""MetaFormer (MetaConv / MetaPool) autograd functions on HIP kernels.

Frame-major convention as in layers.py: a reference (B, C, L) tensor is held as (B*L, C).
The MetaFormer models switch which axis is "time" several times (the decoder runs convs
with time as channels, MetaConv.py:162-179), so explicit batched transposes appear where
the reference's conv axis changes.

References:
  MetaBlock      factory/MetaConv.py:8-76 (conv mixer), factory/MetaPool.py:18-77 (pool mixer)
  GroupNorm(1)   factory/Norm.py:53-60
  PatchEmbed     factory/Norm.py:63-82
  MLPMixer       factory/MLPMixer.py:58-92 (depth 1, expansion 4, dropout 0)
"""
from __future__ import annotations

import contextlib

import torch

from . import kernels as K
from . import layers as Lyr
from .kernels import operand


# gradient-sink mode: the mixer's weight-gradient products (both operands K-strided, compute-bound)
# run on the side stream beside the memory-bound data-gradient chain (LayerNorm, GELU, transposes,
# pads) instead of in line with it (profiles/r3_metaconv_mixer_ab.txt)


def _wside(on, *keep):
    """Context for a weight-gradient product: the side stream (after everything queued so far,
    `keep` alive until join_side) when `on`, else the current stream.  Operand twins must exist
    before entering: a twin made inside would be written on the side stream and read on this one."""
    if not on:
        return contextlib.nullcontext()
    sd = Lyr._Side()
    sd.keep(*keep)
    return sd


def _sink(p):
    """p.grad when the gradient sink is on (TrainStep: kernels accumulate straight into the flat
    gradient buffer and the autograd functions return None for parameters), else None."""
    return Lyr._grad_of(p) if Lyr.sink_on() else None


# ------------------------------------------------------------------------------ elementwise
class _AddFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        return K.add(a, b)

    @staticmethod
    def backward(ctx, g):
        return g, g


def add(a, b):
    return _AddFn.apply(a, b)


class _TransposeFn(torch.autograd.Function):
    """(B, R, C) -> (B, C, R), both stored as 2-D row blocks."""

    @staticmethod
    def forward(ctx, x, B, R, C):
        ctx.dims = (B, R, C)
        return K.transpose_batched(x.contiguous(), B, R, C).view(B * C, R)

    @staticmethod
    def backward(ctx, g):
        B, R, C = ctx.dims
        return K.transpose_batched(g.contiguous(), B, C, R).view(B * R, C), None, None, None


def transpose(x, B, R, C):
    return _TransposeFn.apply(x, B, R, C)


class _GroupNormFn(torch.autograd.Function):
    """GroupNorm(1, C) on frame-major (B*L, C): per-sample statistics over all L*C values."""

    @staticmethod
    def forward(ctx, x, B, gamma, beta, eps, twin):
        C = x.shape[1]
        y, mean, rstd = K.group_norm_fwd(x, B, C, gamma, beta, eps, twin=twin)
        ctx.save_for_backward(x, gamma, mean, rstd)
        ctx.B, ctx.beta = B, beta
        return y

    @staticmethod
    def backward(ctx, g):
        x, gamma, mean, rstd = ctx.saved_tensors
        C = x.shape[1]
        if Lyr.sink_on():
            dx = K.group_norm_bwd(g.contiguous(), x, gamma, mean, rstd, ctx.B, C, _sink(gamma), _sink(ctx.beta),
                                  accumulate=True)
            return dx, None, None, None, None, None
        dgamma = torch.empty(C, device=x.device)
        dbeta = torch.empty(C, device=x.device)
        dx = K.group_norm_bwd(g.contiguous(), x, gamma, mean, rstd, ctx.B, C, dgamma, dbeta)
        return dx, None, dgamma, dbeta, None, None


def group_norm(x, B, gn, twin=False):
    """twin: the output's bf16 operand twin in the same pass (a GEMM reads it next)."""
    return _GroupNormFn.apply(x, B, gn.weight, gn.bias, gn.eps, twin)


class _PoolMixerFn(torch.autograd.Function):
    """Pooling token mixer: AvgPool1d(3, 1, 1, count_include_pad=False)(x) - x (MetaPool.py:7-15)."""

    @staticmethod
    def forward(ctx, x, B, Lf):
        ctx.dims = (B, Lf, x.shape[1])
        return K.pool3_mixer(x, B, Lf, x.shape[1])

    @staticmethod
    def backward(ctx, g):
        B, Lf, C = ctx.dims
        return K.pool3_mixer(g.contiguous(), B, Lf, C, backward=True), None, None


def pool_mixer(x, B, Lf):
    return _PoolMixerFn.apply(x, B, Lf)


# ------------------------------------------------------------------------------ plain conv
class _ConvFn(torch.autograd.Function):
    """Conv1d + bias (stride 1) on frame-major input (PatchEmbed, MLP-Mixer output conv)."""

    @staticmethod
    def forward(ctx, x, cache, B, T_in, pad, w, b):
        Wf, _ = Lyr.conv_packs(cache, w)
        x = K.twin(x)  # bf16 mode: the conv streams its bf16 twin (an fp32 window took the fp32-operand kernel)
        y, T_out = Lyr.conv_fwd(x, B, T_in, w, b, pad, Wf)
        ctx.cache, ctx.args, ctx.bias = cache, (B, T_in, T_out, pad), b
        ctx.save_for_backward(x, w)
        ctx.x16 = getattr(x, "_bf16", None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        K.attach_twin(x, ctx.x16)
        B, T_in, T_out, pad = ctx.args
        dy = K.twin(dy.contiguous())  # both gradient products read dy as a bf16 operand
        sink = Lyr.sink_on()
        dW = Lyr.conv_wgrad(dy, x, B, T_in, T_out, w, pad, into=_sink(w))
        db = K.colsum(dy, B * T_out, w.shape[0], out=_sink(ctx.bias), accumulate=sink)
        dx = None
        if ctx.needs_input_grad[0]:
            _, Wd = Lyr.conv_packs(ctx.cache, w)
            dx = Lyr.conv_dgrad(dy, B, T_in, T_out, w, pad, Wd)
        return (dx, None, None, None, None) + ((None, None) if sink else (dW, db))


def conv(x, conv_mod, cache, B, T_in):
    return _ConvFn.apply(x, cache, B, T_in, conv_mod.padding[0], conv_mod.weight, conv_mod.bias)


class _EncEmbedFn(torch.autograd.Function):
    """cat(mel, c_org broadcast) -> PatchEmbed conv (MetaConv.py:108-112)."""

    @staticmethod
    def forward(ctx, mel2d, emb, cache, B, T, w, b):
        x = K.twin(K.enc_concat(mel2d, emb, B, T))
        Wf, _ = Lyr.conv_packs(cache, w)
        y, _ = Lyr.conv_fwd(x, B, T, w, b, w.shape[-1] // 2, Wf)
        ctx.cache, ctx.args, ctx.n_mel, ctx.bias = cache, (B, T), mel2d.shape[1], b
        ctx.save_for_backward(x, w)
        ctx.x16 = getattr(x, "_bf16", None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        K.attach_twin(x, ctx.x16)
        B, T = ctx.args
        pad = w.shape[-1] // 2
        dy = K.twin(dy.contiguous())
        sink = Lyr.sink_on()
        dW = Lyr.conv_wgrad(dy, x, B, T, T, w, pad, into=_sink(w))
        db = K.colsum(dy, B * T, w.shape[0], out=_sink(ctx.bias), accumulate=sink)
        if sink:
            dW = db = None
        dmel = demb = None
        nm, Cin = ctx.n_mel, x.shape[1]
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            _, Wd = Lyr.conv_packs(ctx.cache, w)
            # a trained c_org (MetaConv_Adjust.py:256) takes the full-width data gradient
            dx = Lyr.conv_dgrad(dy, B, T, T, w, pad, Wd, n_dx=Cin if ctx.needs_input_grad[1] else nm)
            if ctx.needs_input_grad[1]:
                demb = K.segsum(dx[:, nm:], B, T, Cin - nm, ld=Cin)
            dmel = dx[:, :nm] if ctx.needs_input_grad[0] else None
        return dmel, demb, None, None, None, dW, db


def enc_embed(mel2d, emb, proj, cache, B, T):
    return _EncEmbedFn.apply(mel2d, emb, cache, B, T, proj.weight, proj.bias)


# ------------------------------------------------------------------------------ MLP-Mixer
def _pad8(n):
    return (n + 7) // 8 * 8


def _token_mix_weights(mix, w1, w2, NP):
    """(W1^T, W2) as (NPp x 4NPp) and (W1, W2^T) as (4NPp x NPp) zero-padded matrices in the
    compute dtype, NPp = NP rounded up to a multiple of 8 (121 -> 128, 1849 -> 1856 patches),
    rebuilt when w1 / w2 change.  The padding makes every token-mixing operand 8-aligned in K and
    in its row stride, which the bf16 LDS-DMA GEMM kernels need; padded rows / columns are zero,
    so the products over them add nothing.  The (4NPp x NPp) forms are the K-contiguous B
    operands of the per-utterance products UT_b = Y1T_b W1^T (forward) and dUT_b = dRT_b W2
    (backward), so both run on the NT kernel against the transposed activations the step
    already holds, instead of the TT kernel over two K-strided operands."""
    def build():
        dt = K.compute()
        NPp = _pad8(NP)
        w1t = K.pad_cols(K.transpose(w1.view(4 * NP, NP), K.F32), 4 * NPp)   # (NP, 4NPp)
        w2p = K.pad_cols(w2.view(NP, 4 * NP), 4 * NPp)                         # (NP, 4NPp)
        rows = lambda t: K.pad_cols(t.view(1, NP * 4 * NPp), NPp * 4 * NPp, dtype=dt).view(NPp, 4 * NPp)  # noqa: E731
        w1n = K.pad_cols(w1.view(4 * NP, NP), NPp)                             # (4NP, NPp)
        w2t = K.pad_cols(K.transpose(w2.view(NP, 4 * NP), K.F32), NPp)        # (4NP, NPp)
        rows4 = lambda t: K.pad_cols(t.view(1, 4 * NP * NPp), 4 * NPp * NPp, dtype=dt).view(4 * NPp, NPp)  # noqa: E731
        return rows(w1t), rows(w2p), rows4(w1n), rows4(w2t)
    return mix.tm_cache.get([w1, w2], build)


def _cf_weights(mix, we, w3, w4):
    """Patch-embedding and channel-FF weights in the compute dtype (bf16 in bf16 mode, so the
    products take the LDS-DMA bf16 kernels instead of the fp32-operand path), and their transposes:
    the K-contiguous B operands of the data gradients dP = dZ we, dY2 = dU2 w3, dV2 = dZ2 w4
    (MLPMixer.py:16-23,70-76), which as K-strided operands of the untransposed weights took the
    register-staged kernel (3.3 ms per C4 step, profiles/r3_c4_step_breakdown.txt)."""
    def build():
        dt = K.compute()
        return (K.convert(we, dt), K.convert(w3, dt), K.convert(w4, dt), K.transpose(we, dt), K.transpose(w3, dt),
                K.transpose(w4, dt))
    return mix.cf_cache.get([we, w3, w4], build)


def _out_conv_packs(mix, wc):
    """Packs of the mixer output conv Conv1d(NP -> O, k5) with NP zero-padded to a multiple of
    8 (1849 -> 1856 / 121 -> 128 patches): the padded channels meet zero weights, and the
    bf16 LDS-DMA conv / weight-gradient kernels replace the generic path (2.3 ms -> see
    DESIGN.md).  Returns ((Wf, Wd), padded weight) with the padded weight used for shapes."""
    O, NP, Kw = wc.shape
    NPp = (NP + 7) // 8 * 8
    if NPp == NP:
        return Lyr.conv_packs(mix.cache, wc), wc

    def build():
        dt = K.compute()
        wp = K.pad_cols(wc.view(O, NP * Kw), NPp * Kw).view(O, NPp, Kw)
        return K.conv_pack(wp, 0, dt), K.conv_pack(wp, 1, dt), wp
    Wf, Wd, wp = mix.cache.get([wc], build)
    return (Wf, Wd), wp


def _twins(*ts):
    return tuple(getattr(t, "_bf16", None) for t in ts)


def _lin(x, M, N, Kd, w, b=None, residual=None, out=None):
    """y = x (M x Kd, row-major) . w^T (w: N x Kd) + b (+ residual)."""
    y = torch.empty(M, N, device=x.device) if out is None else out
    K.gemm(M, N, Kd, operand(x, Kd), operand(w, Kd), y, bias=b, residual=residual)
    return y


def _gelu_gemm(M, N, Kd, a, b, bias, dev, batch=1):
    """(U, V): U = a . b^T + bias (the pre-activation the backward needs), V = GELU(U) as the next
    GEMM's operand (bf16 only in bf16 mode).  bf16 mode: V comes out of the GEMM's epilogue
    (avc_gemm_desc.c_bf16_act; the ring kernels compute it in the epilogue, other kernels run one
    GELU pass after the GEMM), instead of a separate pass that re-reads U."""
    if K.compute() != K.BF16:
        U = torch.empty(batch * M, N, device=dev)
        K.gemm(M, N, Kd, a, b, U, bias=bias, batch=batch, c_batch_stride=M * N)
        return U, K.gelu_fwd_operand(U)
    if not _vec(Kd, N, a, b):
        # non-vectorisable operands take the generic kernel, which writes fp32 C only: U in fp32,
        # V made from it by the GELU pass (a dim outside the MetaConv / MetaPool shapes)
        U = torch.empty(batch * M, N, device=dev)
        V = torch.empty(batch * M, N, device=dev, dtype=torch.bfloat16)
        K.gemm(M, N, Kd, a, b, U, bias=bias, batch=batch, c_batch_stride=M * N, c_bf16=V, c_bf16_act=K.ACT_GELU)
        return U, V
    # bf16 mode: U is only the backward's GELU' input -- stored in bf16 (avc_gemm_desc.c_pre_bf16)
    U = torch.empty(batch * M, N, device=dev, dtype=torch.bfloat16)
    V = torch.empty(batch * M, N, device=dev, dtype=torch.bfloat16)
    K.gemm(M, N, Kd, a, b, U, bias=bias, batch=batch, c_batch_stride=M * N, c_bf16=V, c_bf16_act=K.ACT_GELU)
    return U, V


def _dgelu_gemm(M, N, Kd, a, b, U, dev, batch=1, bias_grad=None):
    """dU = (a . b^T) * GELU'(U): fp32 (fp32 mode), or bf16 only -- it is read only as the next
    GEMMs' operand -- from the GEMM epilogue (bf16 mode, avc_gemm_desc.act_grad_of).  bias_grad = (out, n, accumulate): out[:n] (+)= the column sums of
    dU, the bias gradient of the GELU's linear layer -- in bf16 mode in the same epilogue
    (avc_gemm_desc.col_sum) instead of a colsum pass that re-reads dU."""
    if K.compute() != K.BF16:
        dU = torch.empty(batch * M, N, device=dev)
        K.gemm(M, N, Kd, a, b, dU, batch=batch, c_batch_stride=M * N)
        dU = K.gelu_bwd_twin(dU, U)
        if bias_grad is not None:
            out, n, acc = bias_grad
            K.colsum(dU, batch * M, n, ld=N, out=out, accumulate=acc)
        return dU
    d16 = torch.empty(batch * M, N, device=dev, dtype=torch.bfloat16)
    kw = {}
    if bias_grad is not None:
        out, n, acc = bias_grad
        if not acc:
            out.zero_()
        kw = dict(col_sum=out, col_sum_n=n)
    if not _vec(Kd, N, a, b):  # generic kernel: an fp32 C, the bf16 copy made from it by the GELU' pass
        dU = torch.empty(batch * M, N, device=dev)
        K.gemm(M, N, Kd, a, b, dU, batch=batch, c_batch_stride=M * N, c_bf16=d16, act_grad_of=U, **kw)
        return d16
    K.gemm(M, N, Kd, a, b, d16, batch=batch, c_batch_stride=M * N, act_grad_of=U, **kw)
    return d16


def _vec(Kd, N, *ops):
    """Whether a product's operands are vectorisable (contiguous dims and row strides multiples of 4
    elements: avc_gemm's fast / ring kernels, which write the bf16-only GELU outputs)."""
    return Kd % 4 == 0 and N % 4 == 0 and all(o.ld % 4 == 0 and o.batch_stride % 4 == 0 for o in ops)


class _MLPMixerFn(torch.autograd.Function):
    """MLPMixer(image C x L (rows = channels of the frame-major input), patch ps, dim D,
    depth 1, out_dim O) -> frame-major (B*D, O)  [reference: (B, O, D)]."""

    @staticmethod
    def forward(ctx, nf, mix, B, Lf, *params):
        (we, be, g1, b1n, w1, bb1, w2, bb2, g2, b2n, w3, bb3, w4, bb4, wc, bc) = params
        C = nf.shape[1]
        ps = mix.ps
        NP = (C // ps) * (Lf // ps)
        D = we.shape[0]
        dev = nf.device
        # (B*NP, ps^2): bf16 mode writes the patches in bf16 directly (read only as GEMM operands)
        P = K.twin(K.patchify(nf, B, Lf, C, ps, out_bf16=K.compute() == K.BF16))
        weC, w3C, w4C, _, _, _ = _cf_weights(mix, we, w3, w4)
        Z = _lin(P, B * NP, D, ps * ps, weC, be)                # (B*NP, D)
        bf = K.compute() == K.BF16  # Y1 / Y2 are read only as bf16 operands: no fp32 copies
        Y1, m1, r1 = K.layer_norm_fwd(Z, g1, b1n, mix.ln_eps[0], out_bf16=bf)
        # token mixing: UT_b (D x 4NP) = Y1_b^T . W1^T + b1   (Conv1d(NP -> 4NP, k1) on (B, NP, D)),
        # as an NT product of the per-utterance transpose Y1T_b (D x NPp) and W1 (4NPp x NPp).
        # Patch counts are zero-padded to NPp (_token_mix_weights): UT / V carry 4NPp columns
        # (padded ones stay 0: zero weights, zero bias, GELU(0) = 0).
        W1T, W2c, W1n, _ = _token_mix_weights(mix, w1, w2, NP)
        NPp = W1T.shape[0]
        # Y1^T per utterance, (B*D, NPp): the K-contiguous A operand of UT_b = Y1T_b W1^T here and
        # the K = B*D operand of the dW1 product (backward)
        Y1T = K.transpose_pad(Y1, B, NP, D, NPp, dtype=K.compute())
        bb1p = K.pad_cols(bb1.view(1, 4 * NP), 4 * NPp).view(-1)
        UT, V = _gelu_gemm(D, 4 * NPp, NPp, operand(Y1T, NPp, batch_stride=D * NPp), operand(W1n, NPp), bb1p, dev,
                           batch=B)
        if bf and D % 4 == 0:
            # Z1 = Z + RT^T per utterance straight from the GEMM epilogue: each D-row block of the
            # (B*D x NP) product stored transposed into the frame-major layout, Z read there as the
            # residual (avc_gemm_desc.c_trans_rows; no RT tensor, no copy of Z, no transpose pass)
            Z1 = torch.empty(B * NP, D, device=dev)
            K.gemm(D, NP, 4 * NPp, operand(V, 4 * NPp, batch_stride=D * 4 * NPp), operand(W2c, 4 * NPp), Z1, bias=bb2,
                   batch=B, c_batch_stride=D * NP, residual=Z, c_trans_rows=D)
        else:
            RT = torch.empty(B * D, NP, device=dev)
            K.gemm(D, NP, 4 * NPp, operand(V, 4 * NPp, batch_stride=D * 4 * NPp), operand(W2c, 4 * NPp), RT,
                   bias=bb2, batch=B, c_batch_stride=D * NP)
            Z1 = K.transpose_batched(RT, B, D, NP, out=K.convert(Z, K.F32), accumulate=True).view(B * NP, D)
        Y2, m2, r2 = K.layer_norm_fwd(Z1, g2, b2n, mix.ln_eps[1], out_bf16=bf)
        U2, V2 = _gelu_gemm(B * NP, 4 * D, D, operand(K.twin(Y2), D), operand(w3C, D), bb3, dev)
        Z2 = _lin(V2, B * NP, D, 4 * D, w4C, bb4, residual=Z1)
        (Wf, _), wp = _out_conv_packs(mix, wc)
        if wp.shape[1] != NP:  # padded patch channels, written once in the compute dtype
            Z2T = K.transpose_pad(Z2, B, NP, D, wp.shape[1], dtype=K.compute())
        else:
            Z2T = K.transpose_batched(Z2, B, NP, D).view(B * D, NP)
        out, _ = Lyr.conv_fwd(Z2T, B, D, wp, bc, wc.shape[-1] // 2, Wf)
        ctx.mix, ctx.dims = mix, (B, Lf, C, ps, NP, D)
        ctx.stats = (m1, r1, m2, r2)
        ctx.save_for_backward(P, Z, Y1T, UT, V, Z1, Y2, U2, V2, Z2T, *params)
        ctx.twins = _twins(P, Y2, V2, V)  # saved tensors come back as new objects: carry the twins
        return out

    @staticmethod
    def backward(ctx, dout):
        (P, Z, Y1T, UT, V, Z1, Y2, U2, V2, Z2T, we, be, g1, b1n, w1, bb1, w2, bb2, g2, b2n, w3, bb3, w4, bb4, wc,
         bc) = ctx.saved_tensors
        mix = ctx.mix
        B, Lf, C, ps, NP, D = ctx.dims
        m1, r1, m2, r2 = ctx.stats
        for t, t16 in zip((P, Y2, V2, V), ctx.twins):
            K.attach_twin(t, t16)
        weC, w3C, w4C, weT, w3T, w4T = _cf_weights(mix, we, w3, w4)
        dev = dout.device
        dout = dout.contiguous()
        pad = wc.shape[-1] // 2
        # output conv (NP -> O, k5) over the D frames
        (_, Wd), wp = _out_conv_packs(mix, wc)
        O, NPp, Kw = wp.shape
        # gradient sink (TrainStep): every parameter gradient below accumulates straight into
        # .grad (GEMM accumulate / atomics, colsum and LayerNorm accumulate, crop_add for the
        # zero-padded products) and the function returns None for the parameters -- no autograd
        # accumulation pass per parameter
        sink = Lyr.sink_on()
        side = sink and Lyr.side_stream() is not None
        dout16 = K.twin(dout)
        with _wside(side, dout, dout16, Z2T, wp):
            if NPp != NP:
                dwc = Lyr.conv_wgrad(dout16, Z2T, B, D, D, wp, pad)
                dwc = (K.crop_add(dwc.view(O, NPp * Kw), _sink(wc).view(O, NP * Kw)) if sink
                       else K.pad_cols(dwc.view(O, NPp * Kw), NP * Kw).view(O, NP, Kw))
            else:
                dwc = Lyr.conv_wgrad(dout16, Z2T, B, D, D, wp, pad, into=_sink(wc))
        dbc = K.colsum(dout, B * D, wc.shape[0], out=_sink(bc), accumulate=sink)
        dZ2T = Lyr.conv_dgrad(dout, B, D, D, wp, pad, Wd, n_dx=NP)
        dZ2 = K.transpose_pad(dZ2T, B, D, NP, D, twin=True)
        M = B * NP
        # channel FF: Z2 = GELU(LN2(Z1) W3^T + b3) W4^T + b4 + Z1
        dw4 = _sink(w4) if sink else torch.empty_like(w4)
        with _wside(side, dZ2, V2):
            K.gemm(D, 4 * D, M, operand(dZ2, D, kstrided=True), operand(V2, 4 * D, kstrided=True), dw4,
                   split_k=K.auto_split_k(D, 4 * D, M), accumulate=sink)
        dbb4 = K.colsum(dZ2, M, D, out=_sink(bb4), accumulate=sink)
        dbb3 = _sink(bb3) if sink else torch.empty(4 * D, device=dev)
        dU2 = _dgelu_gemm(M, 4 * D, D, operand(dZ2, D), operand(w4T, D), U2, dev, bias_grad=(dbb3, 4 * D, sink))
        dw3 = _sink(w3) if sink else torch.empty_like(w3)
        with _wside(side, dU2, Y2):
            K.gemm(4 * D, D, M, operand(dU2, 4 * D, kstrided=True), operand(Y2, D, kstrided=True), dw3,
                   split_k=K.auto_split_k(4 * D, D, M), accumulate=sink)
        dY2 = torch.empty(M, D, device=dev)
        K.gemm(M, D, 4 * D, operand(dU2, 4 * D), operand(w3T, 4 * D), dY2)
        dg2, db2n = (_sink(g2), _sink(b2n)) if sink else (torch.empty(D, device=dev), torch.empty(D, device=dev))
        # bf16 mode: dZ1's row sums come out of the same pass -- dbb2[p] = sum over (b, d) of
        # dRT_b[d][p] = sum over b of rowsum(dZ1)[b*NP + p] -- and the padded bf16 dRT operand is
        # ONE transpose of dZ1 (no fp32 dRT, no colsum / pad passes over it)
        tr = K.compute() == K.BF16 and K.ln_vec(D)
        rs1 = torch.empty(B * NP, device=dev) if tr else None
        dZ1 = K.layer_norm_bwd(dY2, Z1, g2, m2, r2, dg2, db2n, accumulate=sink, residual=dZ2, row_sum=rs1)
        # token FF: Z1 = Z + (GELU(Y1^T W1^T + b1) W2^T + b2)^T   per utterance.  dRT_b = dZ1_b^T is
        # read in place from dZ1 (as the transposed operand), so NP is never a contiguous dimension.
        W1T, W2c, _, W2t = _token_mix_weights(mix, w1, w2, NP)
        NPp = W1T.shape[0]
        # Token-mixing weight gradients sum over utterances AND the D positions: with the
        # per-utterance transposes (B*D rows) that sum is the K dimension of ONE product
        # (K = B*D, both operands K-strided), with no per-utterance slabs to reduce.
        if tr:
            dbb2 = K.colsum(rs1, B, NP, out=_sink(bb2), accumulate=sink)
            dRTp = K.transpose_pad(dZ1, B, NP, D, NPp, dtype=K.BF16)
        else:
            dRT = K.transpose_batched(dZ1, B, NP, D).view(B * D, NP)
            dbb2 = K.colsum(dRT, B * D, NP, out=_sink(bb2), accumulate=sink)
            dRTp = K.pad_cols(dRT, NPp, dtype=K.compute())
        with _wside(side, dRTp, V):
            dW2p = torch.empty(NPp, 4 * NPp, device=dev)
            K.gemm(NPp, 4 * NPp, B * D, operand(dRTp, NPp, kstrided=True), operand(V, 4 * NPp, kstrided=True), dW2p,
                   split_k=K.auto_split_k(NPp, 4 * NPp, B * D))
            dW2 = K.crop_add(dW2p[:NP], _sink(w2).view(NP, 4 * NP)) if sink else K.pad_cols(dW2p, 4 * NP)[:NP]
        dbb1 = _sink(bb1) if sink else torch.empty(4 * NP, device=dev)
        dUT = _dgelu_gemm(D, 4 * NPp, NPp, operand(dRTp, NPp, batch_stride=D * NPp), operand(W2t, NPp), UT, dev,
                          batch=B, bias_grad=(dbb1, 4 * NP, sink))
        with _wside(side, dUT, Y1T):
            dW1p = torch.empty(4 * NPp, NPp, device=dev)
            K.gemm(4 * NPp, NPp, B * D, operand(dUT, 4 * NPp, kstrided=True), operand(Y1T, NPp, kstrided=True),
                   dW1p, split_k=K.auto_split_k(4 * NPp, NPp, B * D))
            dW1 = K.crop_add(dW1p[:4 * NP], _sink(w1).view(4 * NP, NP)) if sink else K.pad_cols(dW1p, NP)[:4 * NP]
        if tr:  # dY1 straight into the frame-major layout (avc_gemm_desc.c_trans_rows)
            dY1 = torch.empty(M, D, device=dev)
            K.gemm(B * D, NP, 4 * NPp, operand(dUT, 4 * NPp), operand(W1T, 4 * NPp), dY1, c_trans_rows=D)
        else:
            dY1T = torch.empty(B * D, NP, device=dev)
            K.gemm(B * D, NP, 4 * NPp, operand(dUT, 4 * NPp), operand(W1T, 4 * NPp), dY1T)
            dY1 = K.transpose_batched(dY1T, B, D, NP).view(M, D)
        dg1, db1n = (_sink(g1), _sink(b1n)) if sink else (torch.empty(D, device=dev), torch.empty(D, device=dev))
        dZ = K.twin(K.layer_norm_bwd(dY1, Z, g1, m1, r1, dg1, db1n, accumulate=sink, residual=dZ1, twin=True))
        # patch embedding
        pp = ps * ps
        dwe = _sink(we) if sink else torch.empty_like(we)
        with _wside(side, dZ, P):
            K.gemm(D, pp, M, operand(dZ, D, kstrided=True), operand(P, pp, kstrided=True), dwe,
                   split_k=K.auto_split_k(D, pp, M), accumulate=sink)
        dbe = K.colsum(dZ, M, D, out=_sink(be), accumulate=sink)
        dnf = None
        if ctx.needs_input_grad[0]:
            dP = torch.empty(M, pp, device=dev)
            K.gemm(M, pp, D, operand(dZ, D), operand(weT, D), dP)
            dnf = K.patchify(dP, B, Lf, C, ps, backward=True)
        if sink:
            return (dnf, None, None, None) + (None,) * 16
        return (dnf, None, None, None, dwe, dbe, dg1, db1n, dW1.view_as(w1), dbb1, dW2.view_as(w2), dbb2, dg2, db2n,
                dw3, dbb3, dw4, dbb4, dwc, dbc)


def mlp_mixer(nf, mixer, B, Lf):
    return _MLPMixerFn.apply(nf, mixer, B, Lf, *mixer.flat_params())
