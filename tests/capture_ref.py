"""Op-level capture of the production (bf16) step, each op checked against fp64 on its OWN inputs.

`Capture` wraps the kernels-module entry points that carry the step's arithmetic -- every GEMM
(conv windows, halo conv / halo dW, split-K weight gradients, the lstm1 fold products, fused
bias / residual / BN-statistics / BN-finalize / bf16-twin / cperm epilogues), the persistent and
wavefront LSTM recurrences (the folded lstm1's included), the small-H BiLSTM, the BN apply / backward passes, the code
expansion, the MetaFormer blocks (GroupNorm, LayerNorm, GELU twins, pooling mixer, patchify,
batched transposes), the discriminator head, the loss block, BCE and the fused Adam.  For each call it synchronises, snapshots what the op accumulates into, runs the
production kernel, and computes the same op in float64 from the very tensors the kernel read
(bf16 operands are exact in fp64).  The deviation recorded per output is the relative
Frobenius norm  ||got - ref|| / ||ref||  (of the increment for accumulating outputs).

The fp64 restatements follow the C-ABI contract in include/autovc_hip.h (avc_operand window /
kstrided / batch semantics, avc_gemm_desc epilogues, avc_lstm_* and avc_bn_* contracts) and
nn.LSTM / nn.BatchNorm1d math (reference factory/AutoVC.py:26-41,43,77,96,110).  Test
infrastructure only: nothing in the product imports this file.
"""
from __future__ import annotations

import contextlib

import torch

from autoformer_amd import kernels as K

ACT_NONE, ACT_RELU, ACT_TANH, ACT_LEAKY, ACT_GELU, ACT_SIGMOID = 0, 1, 2, 3, 4, 5


def _storage_view(t: torch.Tensor):
    """A 1-D tensor over t's whole storage and t's element offset in it."""
    st = t.untyped_storage()
    base = torch.empty(0, dtype=t.dtype, device=t.device)
    base.set_(st, 0, (st.nbytes() // t.element_size(),))
    return base, t.storage_offset()


def materialize(o, R: int, Kd: int, z: int = 0) -> torch.Tensor:
    """The logical R x Kd matrix of one avc_operand (batch index z) in float64."""
    t = o._keep
    assert o.ptr == t.data_ptr(), "operand pointer moved off its tensor"
    base, off = _storage_view(t)
    off += z * o.batch_stride
    if o.taps == 0:
        strides = (1, o.ld) if o.kstrided else (o.ld, 1)
        return base.as_strided((R, Kd), strides, off).double()
    frames, other = (Kd, R) if o.kstrided else (R, Kd)
    assert other == o.taps * o.chans and frames % o.t_out == 0, (R, Kd, o.taps, o.chans, o.t_out)
    nb = frames // o.t_out
    src = base.as_strided((nb, o.t_in, o.chans), (o.t_in * o.ld, o.ld, 1), off).double()
    ti = torch.arange(o.t_out, device=t.device)[:, None] + torch.arange(o.taps, device=t.device)[None, :] - o.pad
    valid = ((ti >= 0) & (ti < o.t_in)).to(torch.float64)
    win = src[:, ti.clamp(0, o.t_in - 1), :] * valid[None, :, :, None]  # (nb, t_out, taps, chans)
    win = win.reshape(frames, other)
    return win.t() if o.kstrided else win


def _rel(got, ref, base=None, floor=0.0):
    """||got - ref|| / max(||ref||, floor) (of the increments over `base` for accumulating outputs).
    `floor` is the natural scale of an output that may vanish: a per-channel sum of a gradient whose
    sum is analytically zero (e.g. the bias gradient of a GroupNorm feeding the zero-mean pooling
    mixer) has only rounding noise left to compare."""
    got = got.double()
    ref = ref.double()
    if base is not None:
        got = got - base
        ref = ref - base
    den = max(ref.norm().item(), floor)
    num = (got - ref).norm().item()
    return num / den if den > 0 else num


def _c_view(c, M, N, ldc, batch, cbs, cperm, ctr=0):
    base, off = _storage_view(c)
    if ctr:  # avc_gemm_desc.c_trans_rows: every ctr-row block of C stored transposed
        nb = batch if cbs else 1
        v = base.as_strided((nb * M // ctr, N, ctr), (N * ctr, ctr, 1), off)
        return v.transpose(1, 2).reshape(nb, M, N)
    if cperm:
        taps = cperm
        v = base.as_strided((M, taps, N // taps), (ldc, 1, taps), off)
        return v.reshape(1, M, N)
    nb = batch if cbs else 1
    return base.as_strided((nb, M, N), (cbs, ldc, 1), off)


def _act(pre, act, slope=0.2):
    if act == ACT_NONE:
        return pre
    if act == ACT_RELU:
        return torch.relu(pre)
    if act == ACT_TANH:
        return torch.tanh(pre)
    if act == ACT_SIGMOID:
        return torch.sigmoid(pre)
    if act == ACT_LEAKY:
        return torch.nn.functional.leaky_relu(pre, slope)
    if act == ACT_GELU:
        return torch.nn.functional.gelu(pre)
    raise ValueError(act)


def _act_grad_from_pre(pre, act, slope=0.2):
    if act == ACT_NONE:
        return torch.ones_like(pre)
    if act == ACT_RELU:
        return (pre > 0).to(pre.dtype)
    if act == ACT_TANH:
        return 1 - torch.tanh(pre) ** 2
    if act == ACT_SIGMOID:
        s = torch.sigmoid(pre)
        return s * (1 - s)
    if act == ACT_LEAKY:
        return torch.where(pre > 0, torch.ones_like(pre), torch.full_like(pre, slope))
    raise ValueError(act)


def edge_class(T, pad, device=None):
    """Edge class of every frame t of an utterance (avc_gemm_desc.row_bias)."""
    t = torch.arange(T, device=device)
    return torch.where(t < pad, t, torch.where(t >= T - pad, 2 * pad - (T - 1 - t), torch.full_like(t, pad)))


def row_bias_rows(S, M, T, pad):
    """The (M, N) float64 matrix the row bias adds: row b*T + t takes S[b*(2 pad + 1) + class(t)]."""
    ncls = 2 * pad + 1
    rows = torch.arange(M, device=S.device)
    idx = (rows // T) * ncls + edge_class(T, pad, S.device)[rows % T]
    return S.double()[idx]


# ----------------------------------------------------------------------------- LSTM fp64
def lstm_fwd_ref(xproj, whh, B, T, H, dirs):
    """nn.LSTM forward of `dirs` directions from the input projections (B*T, dirs*4H) and W_hh
    (dirs*4H, H); gate order i, f, g, o; the reverse direction runs t = T-1 .. 0."""
    X = xproj.double().view(B, T, dirs, 4 * H)
    hs = torch.empty(B, T, dirs, H, dtype=torch.float64, device=xproj.device)
    cs = torch.empty_like(hs)
    gs = torch.empty(B, T, dirs, 4 * H, dtype=torch.float64, device=xproj.device)
    for d in range(dirs):
        W = whh[d * 4 * H:(d + 1) * 4 * H].double()
        h = torch.zeros(B, H, dtype=torch.float64, device=xproj.device)
        c = torch.zeros_like(h)
        for t in (range(T) if d == 0 else range(T - 1, -1, -1)):
            pre = X[:, t, d] + h @ W.t()
            i, f = torch.sigmoid(pre[:, :H]), torch.sigmoid(pre[:, H:2 * H])
            g, o = torch.tanh(pre[:, 2 * H:3 * H]), torch.sigmoid(pre[:, 3 * H:])
            c = f * c + i * g
            h = o * torch.tanh(c)
            hs[:, t, d], cs[:, t, d] = h, c
            gs[:, t, d] = torch.cat([i, f, g, o], 1)
    return hs.reshape(B * T, dirs * H), cs.reshape(B * T, dirs * H), gs.reshape(B * T, dirs * 4 * H)


def lstm_bwd_ref(dh, c, gates, W, B, T, H, dirs):
    """dL/d(pre-activation gates) of `dirs` directions from the upstream dh (B*T, dirs*H), the
    saved cell states and activated gates, and W_hh (dirs*4H, H) in float64."""
    DH = dh.double().view(B, T, dirs, H)
    C = c.double().view(B, T, dirs, H)
    Gt = gates.double().view(B, T, dirs, 4 * H)
    out = torch.empty(B, T, dirs, 4 * H, dtype=torch.float64, device=dh.device)
    for d in range(dirs):
        Wd = W[d * 4 * H:(d + 1) * 4 * H].double()
        dhr = torch.zeros(B, H, dtype=torch.float64, device=dh.device)
        dc = torch.zeros_like(dhr)
        order = range(T - 1, -1, -1) if d == 0 else range(T)
        for t in order:
            tp = t - 1 if d == 0 else t + 1
            cp = C[:, tp, d] if 0 <= tp < T else torch.zeros_like(dc)
            i, f, g, o = (Gt[:, t, d, q * H:(q + 1) * H] for q in range(4))
            dht = DH[:, t, d] + dhr
            tc = torch.tanh(C[:, t, d])
            dcs = dc + dht * o * (1 - tc * tc)
            dG = torch.cat([dcs * g * i * (1 - i), dcs * cp * f * (1 - f), dcs * i * (1 - g * g),
                            dht * tc * o * (1 - o)], 1)
            out[:, t, d] = dG
            dhr = dG @ Wd
            dc = dcs * f
    return out.reshape(B * T, dirs * 4 * H)


class Capture:
    """Context manager: record every wrapped op of the enclosed code with its fp64 deviation.
    `records` = list of (op, shape tag, {output: rel-Frobenius})."""

    def __init__(self, skip_bnb=True):
        self.records = []
        self.skip_bnb = skip_bnb
        self._orig = {}

    # ---------------------------------------------------------------- wrappers
    def _gemm(self, M, N, Kd, a, b, c, ldc=None, bias=None, accumulate=False, split_k=1, bn_partial=None, batch=1,
              c_batch_stride=0, comp=None, c_bf16=None, residual=None, cperm=0, bn_fin=None, bnb=None, row_bias=None,
              c_bf16_act=0, act_grad_of=None, col_sum=None, col_sum_n=0, c_trans_rows=0):
        f = self._orig["gemm"]
        kw = dict(ldc=ldc, bias=bias, accumulate=accumulate, split_k=split_k, bn_partial=bn_partial, batch=batch,
                  c_batch_stride=c_batch_stride, comp=comp, c_bf16=c_bf16, residual=residual, cperm=cperm,
                  bn_fin=bn_fin, bnb=bnb, row_bias=row_bias, c_bf16_act=c_bf16_act, act_grad_of=act_grad_of,
                  col_sum=col_sum, col_sum_n=col_sum_n, c_trans_rows=c_trans_rows)
        if bnb is not None and self.skip_bnb:
            return f(M, N, Kd, a, b, c, **kw)
        torch.cuda.synchronize()
        ldc_ = N if ldc is None else ldc
        only16 = c.dtype == torch.bfloat16 and not c_bf16_act  # (with c_bf16_act: a bf16 pre-activation)
        ctr = c_trans_rows
        cv = _c_view(c, M, N, ldc_, batch, c_batch_stride, cperm, ctr)
        before = cv.double().clone() if accumulate else None
        ncs = (col_sum_n or N) if col_sum is not None else 0
        cs_before = col_sum[:ncs].double().clone() if ncs else None
        # product in fp64 from the operands the kernel reads (bf16 twins in bf16 mode)
        P = None
        for z in range(batch):
            pz = materialize(a, M, Kd, z) @ materialize(b, N, Kd, z).t()
            if c_batch_stride or batch == 1:
                P = pz[None] if P is None else torch.cat([P, pz[None]])
            else:
                P = pz[None] if P is None else P + pz[None]
        if bias is not None:
            P = P + bias.double()[None, None, :N]
        if residual is not None:
            P = P + _c_view(residual, M, N, ldc_, batch, c_batch_stride, 0, ctr).double()
        if row_bias is not None:
            P = P + row_bias_rows(row_bias[0], M, row_bias[1], row_bias[2])[None]
        if act_grad_of is not None:  # the GELU backward folded into the epilogue
            xg = _c_view(act_grad_of, M, N, ldc_, batch, c_batch_stride, 0).double()
            P = P * (0.5 * (1.0 + torch.erf(xg / 2 ** 0.5)) + xg * torch.exp(-0.5 * xg * xg) / (2 * torch.pi) ** 0.5)
        stats = f(M, N, Kd, a, b, c, **kw)
        torch.cuda.synchronize()
        got = _c_view(c, M, N, ldc_, batch, c_batch_stride, cperm, ctr).double()
        ref = P if before is None else before + P
        tag = (f"gemm M{M} N{N} K{Kd}" + (f" b{batch}" if batch > 1 else "") + (f" sk{split_k}" if split_k > 1 else "")
               + (" acc" if accumulate else "") + (" win" if a.taps or b.taps else "") + (" cperm" if cperm else "")
               + (" bf16out" if only16 else "") + (" rowbias" if row_bias is not None else "")
               + (" gelu" if c_bf16_act else "") + (" dgelu" if act_grad_of is not None else "")
               + (" colsum" if ncs else "") + (" trans" if ctr else ""))
        res = {"C": _rel(got, ref, before)}
        if ncs:  # the bias gradient accumulated in the epilogue: column sums of the stored values
            cs_ref = cs_before + ref.reshape(-1, N)[:, :ncs].sum(0)
            res["col_sum"] = _rel(col_sum[:ncs].double(), cs_ref, cs_before)
        if c_bf16 is not None and not only16:
            r16 = torch.nn.functional.gelu(ref) if c_bf16_act else ref
            res["C_bf16"] = _rel(_c_view(c_bf16, M, N, ldc_, batch, c_batch_stride, 0), r16, before)
        if bn_partial is not None:
            # per statistics tile (sum, M2) of the stored values -> column mean / variance; the tiles are
            # 128 rows, or one utterance (a.t_out rows) when the one-utterance halo conv ran
            from autoformer_amd import _lib

            tr = a.t_out if _lib.lib().avc_gemm_ring_last() == 3 else 128
            nt = (M + tr - 1) // tr
            part = bn_partial.double().reshape(-1)[:nt * N * 2].view(nt, N, 2)
            cnt = torch.tensor([min(tr, M - tr * i) for i in range(nt)], dtype=torch.float64, device=c.device)
            mean = part[:, :, 0].sum(0) / M
            tmean = part[:, :, 0] / cnt[:, None]
            var = (part[:, :, 1].sum(0) + (cnt[:, None] * (tmean - mean[None]) ** 2).sum(0)) / M
            rm, rv = ref[0].mean(0), ref[0].var(0, unbiased=False)
            res["bn_mean"] = _rel(mean, rm)
            res["bn_var"] = _rel(var, rv)
            if stats is not None:
                kmean, krstd = stats[0], stats[1]
                res["bn_fin_mean"] = _rel(kmean, rm)
                res["bn_fin_rstd"] = _rel(krstd, 1.0 / torch.sqrt(rv + bn_fin[6]))
        self.records.append(("gemm", tag, res))
        return stats

    def _lstm_fwd(self, xproj, w_hh, B, T, H, dirs, hbuf=None):
        torch.cuda.synchronize()
        h, c, g = self._orig["lstm_fwd"](xproj, w_hh, B, T, H, dirs, hbuf)
        torch.cuda.synchronize()
        rh, rc, rg = lstm_fwd_ref(xproj, w_hh, B, T, H, dirs)
        res = {"h": _rel(h, rh), "c": _rel(c, rc), "gates": _rel(g, rg)}
        if getattr(h, "_bf16", None) is not None:
            res["h_bf16"] = _rel(h._bf16, rh)
        self.records.append(("lstm_fwd", f"lstm_fwd B{B} T{T} H{H} dirs{dirs}", res))
        return h, c, g

    def _lstm2_fwd(self, xproj0, w_hh0, w_ih1, w_hh1, bias1, B, T, H):
        torch.cuda.synchronize()
        outs = self._orig["lstm2_fwd"](xproj0, w_hh0, w_ih1, w_hh1, bias1, B, T, H)
        torch.cuda.synchronize()
        h0, c0, g0 = lstm_fwd_ref(xproj0, w_hh0, B, T, H, 1)
        x1 = h0 @ w_ih1.double().t() + bias1.double()[None]
        h1, c1, g1 = lstm_fwd_ref(x1, w_hh1, B, T, H, 1)
        names = ("h0", "c0", "gates0", "h1", "c1", "gates1")
        res = {n: _rel(o, r) for n, o, r in zip(names, outs, (h0, c0, g0, h1, c1, g1))}
        self.records.append(("lstm2_fwd", f"lstm2_fwd B{B} T{T} H{H}", res))
        return outs

    def _lstm_bwd(self, dh, h, c, g, w_hh, w_hh_t, B, T, H, dirs, gbuf=None):
        torch.cuda.synchronize()
        dg = self._orig["lstm_bwd"](dh, h, c, g, w_hh, w_hh_t, B, T, H, dirs, gbuf)
        torch.cuda.synchronize()
        if w_hh is not None:
            W = w_hh
        else:
            W = torch.cat([w_hh_t[d * H:(d + 1) * H].t() for d in range(dirs)], 0)
        ref = lstm_bwd_ref(dh, c, g, W, B, T, H, dirs)
        res = {"dG": _rel(dg, ref)}
        if getattr(dg, "_bf16", None) is not None:
            res["dG_bf16"] = _rel(dg._bf16, ref)
        self.records.append(("lstm_bwd", f"lstm_bwd B{B} T{T} H{H} dirs{dirs}", res))
        return dg

    def _lstm2_bwd(self, dh1, c0, g0, c1, g1, wt0, wti1, wt1, B, T, H, fp32=True, db=False):
        """The two-layer wavefront backward against the layer-by-layer fp64 reference: layer 1 from
        dh1, layer 0 from dG1 W_ih1 (the dX1 the wavefront forms inside its recurrence); with db, the
        per-group bias-gradient partials against the fp64 dG summed over each 16-utterance group."""
        torch.cuda.synchronize()
        out = self._orig["lstm2_bwd"](dh1, c0, g0, c1, g1, wt0, wti1, wt1, B, T, H, fp32=fp32, db=db)
        torch.cuda.synchronize()
        dg0, dg1 = out[0], out[1]
        ref1 = lstm_bwd_ref(dh1, c1, g1, wt1.t(), B, T, H, 1)
        ref0 = lstm_bwd_ref(ref1 @ wti1.double().t(), c0, g0, wt0.t(), B, T, H, 1)
        res = {}
        if fp32:
            res["dG0"], res["dG1"] = _rel(dg0, ref0), _rel(dg1, ref1)
            dg0, dg1 = dg0._bf16, dg1._bf16
        res["dG0_bf16"], res["dG1_bf16"] = _rel(dg0, ref0), _rel(dg1, ref1)
        if db:
            ng = -(-B // 16)
            for layer, ref in ((0, ref0), (1, ref1)):
                r = torch.zeros(ng * 16, T, 4 * H, dtype=torch.float64, device=ref.device)
                r[:B] = ref.reshape(B, T, 4 * H)
                res[f"db{layer}"] = _rel(out[2][layer], r.view(ng, 16 * T, 4 * H).sum(1))
        self.records.append(("lstm2_bwd", f"lstm2_bwd B{B} T{T} H{H}", res))
        return out

    def _lstm_fwd_fold(self, pcode, nc, w_hh, B, T, H, hbuf):
        """The folded lstm1 forward: step t's projection is row b*nc + t/(T/nc) of pcode."""
        torch.cuda.synchronize()
        h, c, g = self._orig["lstm_fwd_fold"](pcode, nc, w_hh, B, T, H, hbuf)
        torch.cuda.synchronize()
        G = 4 * H
        xproj = pcode.view(B, nc, 1, G).expand(B, nc, T // nc, G).reshape(B * T, G)
        rh, rc, rg = lstm_fwd_ref(xproj, w_hh, B, T, H, 1)
        res = {"h": _rel(h, rh), "c": _rel(c, rc), "gates": _rel(g, rg), "h_bf16": _rel(h._bf16, rh)}
        self.records.append(("lstm_fwd_fold", f"lstm_fwd_fold B{B} T{T} H{H} nc{nc}", res))
        return h, c, g

    def _lstm_bwd_fold(self, dh, c, g, w_hh_t, B, T, H, nc, gbuf=None):
        """The folded lstm1 backward: bf16 dG and the per-code sums S_code (fp32 + bf16 twin)."""
        torch.cuda.synchronize()
        dg16, sc = self._orig["lstm_bwd_fold"](dh, c, g, w_hh_t, B, T, H, nc, gbuf)
        torch.cuda.synchronize()
        ref = lstm_bwd_ref(dh, c, g, w_hh_t.t(), B, T, H, 1)
        rs = ref.view(B * nc, T // nc, 4 * H).sum(1)
        res = {"dG_bf16": _rel(dg16, ref), "s_code": _rel(sc, rs), "s_code_bf16": _rel(sc._bf16, rs)}
        self.records.append(("lstm_bwd_fold", f"lstm_bwd_fold B{B} T{T} H{H} nc{nc}", res))
        return dg16, sc

    def _code_cat(self, codes, emb, B, nc, cd):
        torch.cuda.synchronize()
        out = self._orig["code_cat"](codes, emb, B, nc, cd)
        torch.cuda.synchronize()
        ref = torch.cat([codes.double().reshape(B * nc, cd), emb.double().repeat_interleave(nc, 0)], 1)
        self.records.append(("code_cat", f"code_cat B{B} nc{nc}", {"out": _rel(out, ref)}))
        return out

    def _bn_apply(self, y, scale, shift, act, residual=None, out=None, twin16=None, out_bf16=False):
        torch.cuda.synchronize()
        o = self._orig["bn_apply"](y, scale, shift, act, residual=residual, out=out, twin16=twin16,
                                   out_bf16=out_bf16)
        torch.cuda.synchronize()
        ref = _act(y.double() * scale.double()[None] + shift.double()[None], act)
        if residual is not None:
            ref = ref + residual.double()
        res = {"out": _rel(o, ref)}
        if getattr(o, "_bf16", None) is not None:
            res["out_bf16"] = _rel(o._bf16, ref)
        self.records.append(("bn_apply", f"bn_apply M{y.shape[0]} C{y.shape[1]} act{act}", res))
        return o

    def _bn_bwd(self, dA, a, y, mean, rstd, gamma, act, need_dbias=True, into=None, twin16=None, beta=None,
                dy_bf16=False):
        torch.cuda.synchronize()
        before = [t.double().clone() if t is not None else None for t in into] if into is not None else None
        out = self._orig["bn_bwd"](dA, a, y, mean, rstd, gamma, act, need_dbias=need_dbias, into=into,
                                   twin16=twin16, beta=beta, dy_bf16=dy_bf16)
        torch.cuda.synchronize()
        dy, dgamma, dbeta, _ = out
        yh = (y.double() - mean.double()[None]) * rstd.double()[None]
        gm = gamma.double() if gamma is not None else torch.ones_like(mean, dtype=torch.float64)
        if act == ACT_NONE:
            dz = dA.double()
        elif a is not None and act == ACT_RELU:
            dz = dA.double() * (a.double() > 0)
        elif a is not None and act == ACT_TANH:
            dz = dA.double() * (1 - a.double() ** 2)
        else:
            bt = beta.double() if beta is not None else torch.zeros_like(gm)
            dz = dA.double() * _act_grad_from_pre(yh * gm[None] + bt[None], act)
        M = y.shape[0]
        sdz, sdzy = dz.sum(0), (dz * yh).sum(0)
        rdy = gm[None] * rstd.double()[None] * (dz - sdz[None] / M - yh * sdzy[None] / M)
        res = {"dy": _rel(dy, rdy)}
        if getattr(dy, "_bf16", None) is not None:
            res["dy_bf16"] = _rel(dy._bf16, rdy)
        b0, b1 = (before[0], before[1]) if before is not None else (None, None)
        res["dgamma"] = _rel(dgamma, sdzy + (b0 if b0 is not None else 0), b0)
        res["dbeta"] = _rel(dbeta, sdz + (b1 if b1 is not None else 0), b1)
        self.records.append(("bn_bwd", f"bn_bwd M{M} C{y.shape[1]} act{act}", res))
        return out

    def _expand_codes(self, pc, pe, B, T, nc):
        torch.cuda.synchronize()
        out = self._orig["expand_codes"](pc, pe, B, T, nc)
        torch.cuda.synchronize()
        G = pc.shape[1]
        ref = pc.double().view(B, nc, 1, G).expand(B, nc, T // nc, G).reshape(B, T, G) + pe.double()[:, None, :]
        self.records.append(("expand_codes", f"expand_codes B{B} T{T} nc{nc}", {"out": _rel(out, ref.reshape(B * T, G))}))
        return out

    def _conv_edge_table(self, E, B, Co, Kw, T, pad):
        torch.cuda.synchronize()
        S = self._orig["conv_edge_table"](E, B, Co, Kw, T, pad)
        torch.cuda.synchronize()
        Ev = E.double().view(B, Kw, Co)
        ref = torch.zeros(B, 2 * pad + 1, Co, dtype=torch.float64, device=E.device)
        for cls in range(2 * pad + 1):
            t = cls if cls < pad else (pad if cls == pad else T - 1 - (2 * pad - cls))
            for k in range(Kw):
                if 0 <= t + k - pad < T:
                    ref[:, cls] += Ev[:, k]
        self.records.append(("conv_edge_table", f"conv_edge_table B{B} Co{Co}", {"S": _rel(S, ref.view_as(S))}))
        return S

    def _conv_edge_colsum(self, dy, B, T, C, Kw, pad):
        torch.cuda.synchronize()
        out = self._orig["conv_edge_colsum"](dy, B, T, C, Kw, pad)
        torch.cuda.synchronize()
        d = dy.double().view(B, T, C)
        ref = torch.stack([d[:, max(0, pad - k):min(T, T + pad - k)].sum(1) for k in range(Kw)], 1)
        self.records.append(("conv_edge_colsum", f"conv_edge_colsum B{B} T{T} C{C}", {"Sdy": _rel(out, ref.view_as(out))}))
        return out

    # ---------------------------------------------------------------- MetaFormer (C4) blocks
    def _group_norm_fwd(self, x, B, C, gamma, beta, eps, twin=False):
        torch.cuda.synchronize()
        y, mean, rstd = self._orig["group_norm_fwd"](x, B, C, gamma, beta, eps, twin=twin)
        torch.cuda.synchronize()
        xv = x.double().reshape(B, -1)
        mu, var = xv.mean(1), xv.var(1, unbiased=False)
        rs = 1.0 / torch.sqrt(var + eps)
        ref = ((xv - mu[:, None]) * rs[:, None]).view(B, -1, C)
        if gamma is not None:
            ref = ref * gamma.double() + (beta.double() if beta is not None else 0.0)
        res = {"y": _rel(y, ref.view_as(y)), "mean": _rel(mean, mu), "rstd": _rel(rstd, rs)}
        if getattr(y, "_bf16", None) is not None:
            res["y_bf16"] = _rel(y._bf16, ref.view_as(y))
        self.records.append(("group_norm_fwd", f"group_norm_fwd B{B} S{xv.shape[1]} C{C}" + (" twin" if twin else ""),
                             res))
        return y, mean, rstd

    def _group_norm_bwd(self, dy, x, gamma, mean, rstd, B, C, dgamma=None, dbeta=None, accumulate=False):
        torch.cuda.synchronize()
        b0 = dgamma.double().clone() if (dgamma is not None and accumulate) else None
        b1 = dbeta.double().clone() if (dbeta is not None and accumulate) else None
        dx = self._orig["group_norm_bwd"](dy, x, gamma, mean, rstd, B, C, dgamma, dbeta, accumulate)
        torch.cuda.synchronize()
        xh = (x.double().reshape(B, -1) - mean.double()[:, None]) * rstd.double()[:, None]
        g = dy.double().reshape(B, -1)
        gm = gamma.double() if gamma is not None else torch.ones(C, dtype=torch.float64, device=x.device)
        dxh = (g.view(B, -1, C) * gm).reshape(B, -1)
        rdx = rstd.double()[:, None] * (dxh - dxh.mean(1, keepdim=True) - xh * (dxh * xh).mean(1, keepdim=True))
        res = {"dx": _rel(dx, rdx.view_as(dx))}
        fl = 1e-3 * g.norm().item()  # scale of a per-channel sum of g
        if dgamma is not None:
            rg = (g * xh).view(-1, C).sum(0)
            res["dgamma"] = _rel(dgamma, rg + (b0 if b0 is not None else 0), b0, fl)
        if dbeta is not None:
            rb = g.view(-1, C).sum(0)
            res["dbeta"] = _rel(dbeta, rb + (b1 if b1 is not None else 0), b1, fl)
        self.records.append(("group_norm_bwd", f"group_norm_bwd B{B} C{C}", res))
        return dx

    def _layer_norm_fwd(self, x, gamma, beta, eps, out_bf16=False):
        torch.cuda.synchronize()
        y, mean, rstd = self._orig["layer_norm_fwd"](x, gamma, beta, eps, out_bf16=out_bf16)
        torch.cuda.synchronize()
        xv = x.double()
        mu, var = xv.mean(1), xv.var(1, unbiased=False)
        rs = 1.0 / torch.sqrt(var + eps)
        ref = (xv - mu[:, None]) * rs[:, None]
        if gamma is not None:
            ref = ref * gamma.double()[None] + (beta.double()[None] if beta is not None else 0.0)
        res = {"y": _rel(y, ref), "mean": _rel(mean, mu), "rstd": _rel(rstd, rs)}
        self.records.append(("layer_norm_fwd", f"layer_norm_fwd R{x.shape[0]} D{x.shape[1]}" + (" bf16out" if out_bf16
                                                                                               else ""), res))
        return y, mean, rstd

    def _layer_norm_bwd(self, dy, x, gamma, mean, rstd, dgamma=None, dbeta=None, accumulate=False, residual=None,
                        twin=False, row_sum=None):
        torch.cuda.synchronize()
        b0 = dgamma.double().clone() if (dgamma is not None and accumulate) else None
        b1 = dbeta.double().clone() if (dbeta is not None and accumulate) else None
        dx = self._orig["layer_norm_bwd"](dy, x, gamma, mean, rstd, dgamma, dbeta, accumulate, residual=residual,
                                          twin=twin, row_sum=row_sum)
        torch.cuda.synchronize()
        xh = (x.double() - mean.double()[:, None]) * rstd.double()[:, None]
        g = dy.double()
        dxh = g * (gamma.double()[None] if gamma is not None else 1.0)
        rdx = rstd.double()[:, None] * (dxh - dxh.mean(1, keepdim=True) - xh * (dxh * xh).mean(1, keepdim=True))
        if residual is not None:
            rdx = rdx + residual.double()
        res = {"dx": _rel(dx, rdx)}
        if getattr(dx, "_bf16", None) is not None:
            res["dx_bf16"] = _rel(dx._bf16, rdx)
        if row_sum is not None:
            res["row_sum"] = _rel(row_sum, rdx.sum(1), None, 1e-3 * rdx.norm().item())
        fl = 1e-3 * g.norm().item()
        if dgamma is not None:
            res["dgamma"] = _rel(dgamma, (g * xh).sum(0) + (b0 if b0 is not None else 0), b0, fl)
        if dbeta is not None:
            res["dbeta"] = _rel(dbeta, g.sum(0) + (b1 if b1 is not None else 0), b1, fl)
        self.records.append(("layer_norm_bwd", f"layer_norm_bwd R{x.shape[0]} D{x.shape[1]}"
                             + (" res" if residual is not None else "") + (" twin" if twin else ""), res))
        return dx

    def _gelu_fwd_operand(self, x):
        torch.cuda.synchronize()
        y = self._orig["gelu_fwd_operand"](x)
        torch.cuda.synchronize()
        self.records.append(("gelu_fwd", f"gelu_fwd n{x.numel()}",
                             {"y": _rel(y, torch.nn.functional.gelu(x.double()))}))
        return y

    def _gelu_bwd_twin(self, g, x):
        torch.cuda.synchronize()
        dx = self._orig["gelu_bwd_twin"](g, x)
        torch.cuda.synchronize()
        xd = x.double()
        cdf = 0.5 * (1.0 + torch.erf(xd / 2 ** 0.5))
        pdf = torch.exp(-0.5 * xd * xd) / (2 * torch.pi) ** 0.5
        ref = g.double() * (cdf + xd * pdf)
        res = {"dx": _rel(dx, ref)}
        if getattr(dx, "_bf16", None) is not None:
            res["dx_bf16"] = _rel(dx._bf16, ref)
        self.records.append(("gelu_bwd", f"gelu_bwd n{x.numel()}", res))
        return dx

    def _pool3_mixer(self, x, B, Lf, C, backward=False):
        torch.cuda.synchronize()
        xs = x.double().view(B, Lf, C).clone()  # before the kernel: nothing may change it meanwhile
        y = self._orig["pool3_mixer"](x, B, Lf, C, backward)
        torch.cuda.synchronize()
        t = torch.arange(Lf, device=x.device)
        cnt = (1 + (t > 0).to(torch.float64) + (t < Lf - 1).to(torch.float64))[None, :, None]  # window size
        z = torch.zeros(B, 1, C, dtype=torch.float64, device=x.device)
        if not backward:  # y[t] = mean(x[t-1..t+1] inside [0, L)) - x[t]
            ref = (torch.cat([z, xs[:, :-1]], 1) + xs + torch.cat([xs[:, 1:], z], 1)) / cnt - xs
        else:  # the adjoint: dx[s] = sum over windows t containing s of dy[t] / cnt(t) - dy[s]
            q = xs / cnt
            ref = torch.cat([z, q[:, :-1]], 1) + q + torch.cat([q[:, 1:], z], 1) - xs
        self.records.append(("pool3", f"pool3 B{B} L{Lf} C{C}" + (" bwd" if backward else ""),
                             {"y": _rel(y, ref.reshape_as(y))}))
        return y

    def _patchify(self, src, B, Lf, C, ps, backward=False, out_bf16=False):
        torch.cuda.synchronize()
        dst = self._orig["patchify"](src, B, Lf, C, ps, backward, out_bf16)
        torch.cuda.synchronize()
        H, W = C // ps, Lf // ps
        if not backward:  # P[b][h*W + w][p1*ps + p2] = nf[b][w*ps + p2][h*ps + p1]
            ref = src.double().view(B, W, ps, H, ps).permute(0, 3, 1, 4, 2).reshape_as(dst)
        else:
            ref = src.double().view(B, H, W, ps, ps).permute(0, 2, 4, 1, 3).reshape_as(dst)
        if dst.dtype == torch.bfloat16:
            ref = ref.to(torch.bfloat16)  # the bf16 form is the rounding of the same rearrangement
        self.records.append(("patchify", f"patchify B{B} L{Lf} C{C}" + (" bwd" if backward else "")
                             + (" bf16" if dst.dtype == torch.bfloat16 else ""),
                             {"out": _rel(dst, ref)}))
        return dst

    def _transpose_batched(self, src, B, R, C, out=None, accumulate=False):
        torch.cuda.synchronize()
        before = out.double().clone() if (out is not None and accumulate) else None
        dst = self._orig["transpose_batched"](src, B, R, C, out, accumulate)
        torch.cuda.synchronize()
        ref = src.double().reshape(B, R, C).transpose(1, 2).reshape(-1)
        if before is not None:
            ref = ref + before.reshape(-1)
        self.records.append(("btranspose", f"btranspose B{B} R{R} C{C}" + (" acc" if accumulate else ""),
                             {"out": _rel(dst.reshape(-1), ref, None if before is None else before.reshape(-1))}))
        return dst

    def _transpose_pad(self, src, B, R, C, ld, dtype=K.F32, twin=False):
        torch.cuda.synchronize()
        out = self._orig["transpose_pad"](src, B, R, C, ld, dtype, twin)
        torch.cuda.synchronize()
        ref = torch.zeros(B, C, ld, dtype=torch.float64, device=src.device)
        ref[:, :, :R] = src.double().reshape(B, R, C).transpose(1, 2)
        ref = ref.reshape(B * C, ld)
        res = {"out": _rel(out, ref)}
        if getattr(out, "_bf16", None) is not None:
            res["out_bf16"] = _rel(out._bf16, ref)
        self.records.append(("btranspose", f"transpose_pad B{B} R{R} C{C} ld{ld}", res))
        return out

    # ---------------------------------------------------------------- discriminator head (C5)
    def _disc_dense_fwd(self, a, w, bias, B, nl, nc):
        torch.cuda.synchronize()
        p = self._orig["disc_dense_fwd"](a, w, bias, B, nl, nc)
        torch.cuda.synchronize()
        wb = w.double().reshape(nc, nl).t().reshape(-1)  # bin-major order of the channel-major weight
        z = a.double().reshape(B, nl * nc) @ wb + (bias.double().reshape(-1) if bias is not None else 0.0)
        self.records.append(("disc_dense_fwd", f"disc_dense_fwd B{B} L{nl} C{nc}",
                             {"p": _rel(p.reshape(-1), torch.sigmoid(z))}))
        return p

    def _disc_dense_bwd(self, dp, p, a, w, B, nl, nc):
        torch.cuda.synchronize()
        da, dw, db = self._orig["disc_dense_bwd"](dp, p, a, w, B, nl, nc)
        torch.cuda.synchronize()
        pd = p.double().reshape(-1)
        dz = dp.double().reshape(-1) * pd * (1 - pd)
        wb = w.double().reshape(nc, nl).t().reshape(-1)
        rda = dz[:, None] * wb[None]
        rdw = (dz[:, None] * a.double().reshape(B, nl * nc)).sum(0).reshape(nl, nc).t().reshape(-1)
        res = {"da": _rel(da, rda.view_as(da)), "dw": _rel(dw.reshape(-1), rdw), "db": _rel(db.reshape(-1), dz.sum()[None])}
        self.records.append(("disc_dense_bwd", f"disc_dense_bwd B{B} L{nl} C{nc}", res))
        return da, dw, db

    # ---------------------------------------------------------------- losses and the optimizer
    def _vc_loss(self, x, y1, y2, ca, cb, lambda_cd):
        torch.cuda.synchronize()
        out = self._orig["vc_loss"](x, y1, y2, ca, cb, lambda_cd)
        torch.cuda.synchronize()
        m1 = ((x.double() - y1.double()) ** 2).mean()
        m2 = ((x.double() - y2.double()) ** 2).mean()
        l1 = (ca.double() - cb.double()).abs().mean()
        ref = torch.stack([m1, m2, l1, m1 + m2 + lambda_cd * l1])
        self.records.append(("vc_loss", f"vc_loss n{x.numel()} nc{ca.numel()}", {"out": _rel(out, ref)}))
        return out

    def _vc_loss_grad(self, x, y1, y2, ca, cb, lambda_cd, d, need):
        torch.cuda.synchronize()
        outs = self._orig["vc_loss_grad"](x, y1, y2, ca, cb, lambda_cd, d, need)
        torch.cuda.synchronize()
        dv = [float(t.item()) if t is not None else 0.0 for t in d]
        n1, n2 = x.numel(), ca.numel()
        c_id, c_ps, c_cd = dv[3] + dv[0], dv[3] + dv[1], lambda_cd * dv[3] + dv[2]
        ga = c_cd * torch.sign(ca.double() - cb.double()) / n2
        refs = (c_id * 2 * (y1.double() - x.double()) / n1, c_ps * 2 * (y2.double() - x.double()) / n1, ga, -ga)
        res = {n: _rel(o, r) for n, o, r in zip(("g1", "g2", "ga", "gb"), outs, refs) if o is not None}
        self.records.append(("vc_loss_grad", f"vc_loss_grad n{n1}", res))
        return outs

    def _bce_loss(self, p, target):
        torch.cuda.synchronize()
        out = self._orig["bce_loss"](p, target)
        torch.cuda.synchronize()
        pd = p.double()
        ref = -(target * torch.clamp(torch.log(pd), min=-100) + (1 - target) * torch.clamp(torch.log(1 - pd), min=-100))
        self.records.append(("bce_loss", f"bce_loss n{p.numel()} t{target}", {"out": _rel(out, ref.mean())}))
        return out

    def _bce_grad(self, p, target, dloss, through_sigmoid=False):
        torch.cuda.synchronize()
        g = self._orig["bce_grad"](p, target, dloss, through_sigmoid)
        torch.cuda.synchronize()
        pd = p.double()
        ref = dloss.double().reshape(()) * (pd - target) / torch.clamp((1 - pd) * pd, min=1e-12) / p.numel()
        if through_sigmoid:
            ref = ref * pd * (1 - pd)
        self.records.append(("bce_grad", f"bce_grad n{p.numel()}", {"g": _rel(g, ref)}))
        return g

    def _adam(self, p, g, m, v, lr, beta1, beta2, eps, state, advance=True, max_blocks=0):
        torch.cuda.synchronize()
        p0, m0, v0, st0 = p.double().clone(), m.double().clone(), v.double().clone(), state.double().clone()
        self._orig["adam"](p, g, m, v, lr, beta1, beta2, eps, state, advance, max_blocks)
        torch.cuda.synchronize()
        step = float(st0[0].item()) + (1.0 if advance else 0.0)
        gd = g.double()
        rm = beta1 * m0 + (1 - beta1) * gd
        rv = beta2 * v0 + (1 - beta2) * gd * gd
        bc1, bc2 = 1 - beta1 ** step, 1 - beta2 ** step
        rp = p0 - (lr / bc1) * rm / (torch.sqrt(rv) / bc2 ** 0.5 + eps)
        res = {"dp": _rel(p, rp, p0), "m": _rel(m, rm), "v": _rel(v, rv)}
        self.records.append(("adam", f"adam n{p.numel()}" + ("" if advance else " slice"), res))

    # ---------------------------------------------------------------- context
    def __enter__(self):
        for name in ("gemm", "lstm_fwd", "lstm2_fwd", "lstm_bwd", "lstm2_bwd", "lstm_fwd_fold", "lstm_bwd_fold", "code_cat",
                     "bn_apply", "bn_bwd", "expand_codes",
                     "conv_edge_table", "conv_edge_colsum", "group_norm_fwd", "group_norm_bwd", "layer_norm_fwd",
                     "layer_norm_bwd", "gelu_fwd_operand", "gelu_bwd_twin", "pool3_mixer", "patchify",
                     "transpose_batched", "transpose_pad", "disc_dense_fwd", "disc_dense_bwd", "vc_loss", "vc_loss_grad", "bce_loss",
                     "bce_grad", "adam"):
            self._orig[name] = getattr(K, name)
            setattr(K, name, getattr(self, "_" + name))
        return self

    def __exit__(self, *exc):
        for name, f in self._orig.items():
            setattr(K, name, f)
        return False

    # ---------------------------------------------------------------- report
    def worst(self):
        out = []
        for op, tag, res in self.records:
            for k, v in res.items():
                out.append((v, op, tag, k))
        return sorted(out, key=lambda r: -r[0])

    def summary(self, n=15):
        from collections import Counter

        cnt = Counter(op for op, _, _ in self.records)
        lines = [f"{len(self.records)} ops captured: " + ", ".join(f"{k} {v}" for k, v in sorted(cnt.items()))]
        for v, op, tag, k in self.worst()[:n]:
            lines.append(f"  {v:.3e}  {tag} [{k}]")
        return "\n".join(lines)


@contextlib.contextmanager
def captured(**kw):
    cap = Capture(**kw)
    with cap:
        yield cap
