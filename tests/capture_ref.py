"""Op-level capture of the production (bf16) step, each op checked against fp64 on its OWN inputs.

`Capture` wraps the kernels-module entry points that carry the step's arithmetic -- every GEMM
(conv windows, halo conv / halo dW, split-K weight gradients, the lstm1 fold products, fused
bias / residual / BN-statistics / BN-finalize / bf16-twin / cperm epilogues), the persistent and
wavefront LSTM recurrences, the small-H BiLSTM, the BN apply / backward passes and the code
expansion.  For each call it synchronises, snapshots what the op accumulates into, runs the
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


def _rel(got, ref, base=None):
    got = got.double()
    ref = ref.double()
    if base is not None:
        got = got - base
        ref = ref - base
    den = ref.norm().item()
    num = (got - ref).norm().item()
    return num / den if den > 0 else num


def _c_view(c, M, N, ldc, batch, cbs, cperm):
    base, off = _storage_view(c)
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
              c_batch_stride=0, comp=None, c_bf16=None, residual=None, cperm=0, bn_fin=None, bnb=None, row_bias=None):
        f = self._orig["gemm"]
        kw = dict(ldc=ldc, bias=bias, accumulate=accumulate, split_k=split_k, bn_partial=bn_partial, batch=batch,
                  c_batch_stride=c_batch_stride, comp=comp, c_bf16=c_bf16, residual=residual, cperm=cperm,
                  bn_fin=bn_fin, bnb=bnb, row_bias=row_bias)
        if bnb is not None and self.skip_bnb:
            return f(M, N, Kd, a, b, c, **kw)
        torch.cuda.synchronize()
        ldc_ = N if ldc is None else ldc
        only16 = c.dtype == torch.bfloat16
        cv = _c_view(c, M, N, ldc_, batch, c_batch_stride, cperm)
        before = cv.double().clone() if accumulate else None
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
            P = P + _c_view(residual, M, N, ldc_, batch, c_batch_stride, 0).double()
        if row_bias is not None:
            P = P + row_bias_rows(row_bias[0], M, row_bias[1], row_bias[2])[None]
        stats = f(M, N, Kd, a, b, c, **kw)
        torch.cuda.synchronize()
        got = _c_view(c, M, N, ldc_, batch, c_batch_stride, cperm).double()
        ref = P if before is None else before + P
        tag = (f"gemm M{M} N{N} K{Kd}" + (f" b{batch}" if batch > 1 else "") + (f" sk{split_k}" if split_k > 1 else "")
               + (" acc" if accumulate else "") + (" win" if a.taps or b.taps else "") + (" cperm" if cperm else "")
               + (" bf16out" if only16 else "") + (" rowbias" if row_bias is not None else ""))
        res = {"C": _rel(got, ref, before)}
        if c_bf16 is not None and not only16:
            res["C_bf16"] = _rel(_c_view(c_bf16, M, N, ldc_, batch, c_batch_stride, 0), ref, before)
        if bn_partial is not None:
            # per 128-row tile (sum, M2) of the stored values -> column mean / variance
            nt = (M + 127) // 128
            part = bn_partial.double().view(nt, N, 2)
            cnt = torch.tensor([min(128, M - 128 * i) for i in range(nt)], dtype=torch.float64, device=c.device)
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

    # ---------------------------------------------------------------- context
    def __enter__(self):
        for name in ("gemm", "lstm_fwd", "lstm2_fwd", "lstm_bwd", "bn_apply", "bn_bwd", "expand_codes",
                     "conv_edge_table", "conv_edge_colsum"):
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
