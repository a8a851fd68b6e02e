"""Thin, validated Python wrappers over the C-ABI (include/autovc_hip.h).

Every function takes torch tensors that already live on the HIP device, checks shapes /
dtypes / contiguity on the host, and launches on torch's current stream.  No function
here has a CPU fallback.
"""
from __future__ import annotations

import math
import os

import torch

from . import _lib as L
from ._lib import ACT_GELU, ACT_LEAKY, ACT_NONE, ACT_RELU, ACT_SIGMOID, ACT_TANH, BF16, F32  # noqa: F401

_COMPUTE = {"bf16": BF16, "fp32": F32}[os.environ.get("AUTOVC_COMPUTE", "bf16")]


def set_compute(name: str) -> None:
    """'bf16' (bf16 MFMA, fp32 accumulate/state) or 'fp32' (exact fp32 MFMA, parity mode)."""
    global _COMPUTE
    _COMPUTE = {"bf16": BF16, "fp32": F32}[name]


_DETERMINISTIC = False


def set_deterministic(on: bool) -> None:
    """Run-to-run bitwise reproducible gradients (tests): every GEMM without split-K, so no output
    is a sum of float atomics in arrival order.  Slower weight-gradient products; off by default."""
    global _DETERMINISTIC
    _DETERMINISTIC = bool(on)


def compute() -> int:
    return _COMPUTE


def compute_torch_dtype():
    return torch.bfloat16 if _COMPUTE == BF16 else torch.float32


_raw_stream = torch._C._cuda_getCurrentRawStream
_cur_device = torch._C._cuda_getDevice


def stream() -> int:
    """Raw handle of torch's current stream on the current device (every launch goes there).
    The direct C binding: torch.cuda.current_stream() costs ~9 us of Python per call, about
    1 ms of host time per AutoVC step at ~130 launches."""
    return _raw_stream(_cur_device())


def _ptr(t):
    return t.data_ptr() if t is not None else None


def _dt(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.bfloat16:
        return BF16
    raise TypeError(f"unsupported dtype {t.dtype}")


def _dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("autoformer_amd kernels need HIP device tensors (no CPU fallback)")


def require_device(*ts):
    """Model entry points: every tensor argument on the HIP device, or a RuntimeError here -- a host
    pointer reaching a kernel faults the GPU instead of raising."""
    _dev(*(t for t in ts if isinstance(t, torch.Tensor)))


# ------------------------------------------------------------------------- GEMM
def operand(t: torch.Tensor, ld: int, kstrided: bool = False, window=None, batch_stride: int = 0) -> L.Operand:
    """window = (taps, pad, t_out, t_in, chans) or None."""
    _dev(t)
    if _COMPUTE == BF16 and t.dtype == torch.float32:
        tw = getattr(t, "_bf16", None)
        if tw is not None:
            t = tw
    o = L.Operand()
    o._keep = t  # the descriptor holds a raw pointer: keep the tensor alive until launch
    o.ptr = t.data_ptr()
    o.dtype = _dt(t)
    o.kstrided = int(kstrided)
    o.ld = int(ld)
    o.batch_stride = int(batch_stride)
    if window is not None:
        o.taps, o.pad, o.t_out, o.t_in, o.chans = (int(v) for v in window)
    return o


def gemm(M, N, K, a: L.Operand, b: L.Operand, c: torch.Tensor, ldc=None, bias=None, accumulate=False, split_k=1,
         bn_partial=None, batch=1, c_batch_stride=0, comp=None, c_bf16=None, residual=None, cperm=0, bn_fin=None,
         bnb=None, row_bias=None, c_bf16_act=0, act_grad_of=None, col_sum=None, col_sum_n=0, c_trans_rows=0,
         bn_apply=None, bnb_dy=None):
    """cperm = taps > 1: C's columns are (tap, channel) pairs written in nn.Conv1d's [Co][Ci][K]
    weight layout (a conv weight gradient straight into .grad).
    bn_fin = (gamma, beta, running_mean, running_var, nbt, momentum, eps, nupd): the BatchNorm
    finalize of bn_partial fused into the GEMM (avc_gemm_bn); returns (mean, rstd, scale, shift).
    bnb = (y, mean, rstd, gamma, beta, act, coef, dgamma, dbeta, dbias, accumulate): C is dL/da of
    the conv + BN + act layer whose conv output is y; the GEMM also computes that layer's BN
    backward statistics (avc_gemm_bnb: coef[6][N] and the parameter gradients).
    row_bias = (S, T, pad): S[(b*(2 pad + 1) + edge class)][N] added to row b*T + t (the conv0 fold).
    c_bf16_act = ACT_GELU: c_bf16 receives GELU(C), C itself (the pre-activation) is stored to c --
    fp32, or bf16 (avc_gemm_desc.c_pre_bf16) when c is a bf16 tensor; act_grad_of = x (fp32 or
    bf16): C *= GELU'(x) -- the MLP-Mixer GELU forward / backward folded into the GEMM epilogue.
    col_sum: col_sum[:col_sum_n or N] += column sums of C (a bias gradient, float atomics).
    c_trans_rows = R: every R-row block of C stored transposed (avc_gemm_desc.c_trans_rows).
    bn_apply = (out16, act) with bn_fin: act(y*scale + shift) into the bf16 out16 as well (avc_bn_fin.apply_bf16);
    bnb_dy = dy16 with bnb: the producing layer's dy into the bf16 dy16 as well (avc_bnb_args.dy_bf16) --
    fused into the halo conv's epilogue where it runs, a pass after the GEMM otherwise."""
    # every pointer argument must be device memory (operands are checked by operand()); a CPU
    # tensor would reach the kernel as a host pointer and fault the GPU instead of raising here
    _dev(c, bias, residual, c_bf16, bn_partial)
    if _DETERMINISTIC:
        split_k = 1
    pre16 = None
    if c.dtype == torch.bfloat16 and c_bf16_act:  # bf16 pre-activation + bf16 activation
        assert c_bf16 is not None
        c, pre16 = None, c
    elif c.dtype == torch.bfloat16:  # bf16-only output
        assert c_bf16 is None and not accumulate and split_k == 1 and not cperm
        c, c_bf16 = None, c
    else:
        assert c.dtype == torch.float32
    # (a fresh ctypes struct is zeroed: only the fields that differ from 0 / NULL are set -- each
    # field store is ~0.2 us of host time, ~85 GEMMs per AutoVC step)
    d = L.GemmDesc()
    d.M, d.N, d.K, d.batch = int(M), int(N), int(K), int(batch)
    d.a, d.b = a, b
    if c is not None:
        d.c = c.data_ptr()
    d.ldc = int(N if ldc is None else ldc)
    if c_batch_stride:
        d.c_batch_stride = int(c_batch_stride)
    if bias is not None:
        d.bias = bias.data_ptr()
    if accumulate:
        d.accumulate = 1
    d.split_k = int(split_k)
    if bn_partial is not None:
        d.bn_partial = bn_partial.data_ptr()
    d.compute = _COMPUTE if comp is None else comp
    if c_bf16 is not None:
        d.c_bf16 = c_bf16.data_ptr()
    if residual is not None:
        d.residual = residual.data_ptr()
    if cperm:
        d.cperm = int(cperm)
    if c_bf16_act:
        d.c_bf16_act = int(c_bf16_act)
    if col_sum is not None:
        _dev(col_sum)
        d.col_sum, d.col_sum_n = col_sum.data_ptr(), int(col_sum_n)
    if act_grad_of is not None:
        _dev(act_grad_of)
        assert act_grad_of.dtype in (torch.float32, torch.bfloat16)
        d.act_grad_of = act_grad_of.data_ptr()
        d.act_grad_dtype = _dt(act_grad_of)
    if pre16 is not None:
        d.c_pre_bf16 = pre16.data_ptr()
    if c_trans_rows:
        d.c_trans_rows = int(c_trans_rows)
    if row_bias is not None:
        rb, rb_t, rb_pad = row_bias
        _dev(rb)
        d.row_bias, d.rb_t, d.rb_pad = rb.data_ptr(), int(rb_t), int(rb_pad)
    if bnb is not None:
        y, mean, rstd, gamma, beta, act, coef, dgamma, dbeta, dbias, acc = bnb
        _dev(y, mean, rstd, coef)
        bb = L.BnbArgs()
        bb.y, bb.y_dtype, bb.mean, bb.rstd = y.data_ptr(), _dt(y), mean.data_ptr(), rstd.data_ptr()
        bb.gamma, bb.beta, bb.act, bb.coef = _ptr(gamma), _ptr(beta), int(act), coef.data_ptr()
        bb.dgamma, bb.dbeta, bb.dbias, bb.accumulate = _ptr(dgamma), _ptr(dbeta), _ptr(dbias), int(acc)
        ws = torch.empty(int(L.lib().avc_gemm_bnb_ws(int(M), int(N))), device=y.device)
        bb.ws = ws.data_ptr()
        if bnb_dy is not None:
            _dev(bnb_dy)
            assert bnb_dy.dtype == torch.bfloat16 and bnb_dy.shape == (M, N)
            bb.dy_bf16 = bnb_dy.data_ptr()
        L.call("avc_gemm_bnb", d, bb, stream())
        return None
    if bn_fin is None:
        L.call("avc_gemm", d, stream())
        return None
    gamma, beta, rmean, rvar, nbt, momentum, eps, nupd = bn_fin
    dev = bn_partial.device
    stats = tuple(torch.empty(int(N), device=dev) for _ in range(4))
    f = L.BnFin()
    f.gamma, f.beta, f.running_mean, f.running_var, f.num_batches_tracked = (_ptr(gamma), _ptr(beta), _ptr(rmean),
                                                                            _ptr(rvar), _ptr(nbt))
    f.momentum, f.eps, f.nupd = float(momentum), float(eps), int(nupd)
    f.mean, f.rstd, f.scale, f.shift = (t.data_ptr() for t in stats)
    if bn_apply is not None:
        out16, act = bn_apply
        _dev(out16)
        assert out16.dtype == torch.bfloat16 and out16.shape == (M, N)
        f.apply_bf16, f.apply_act = out16.data_ptr(), int(act)
    L.call("avc_gemm_bn", d, f, stream())
    return stats


_TT_SPLITK_MAX = int(os.environ.get("AVC_TT_SPLITK", "8") or 0)


def tt_splitk_reduced(split_k):
    """Whether a split-K weight-gradient (TT) product with this split reduces its partials in the
    kernel (the last-arriving split adds them: gemm_internal.h splitk_last) rather than by atomics
    into a zeroed C.  Mirrors gemm_tt.hip's AVC_TT_SPLITK bound (default 8)."""
    return 1 < split_k <= _TT_SPLITK_MAX


# workgroups a split-K product aims for (~1.5 per CU; re-measured with the in-kernel reduction in round 5)
_SPLIT_TARGET = 384


def auto_split_k(M, N, K, target=None, min_k=256, tiles=None):
    """Split-K factor for the weight-gradient GEMMs (K = frames): about `target` workgroups
    over the 128x128 output tiles (1.5 per CU: a K-loop alone is latency-bound, ~1.4 us per
    64-deep step), each split at least `min_k` long.  Chosen from a split-K sweep of every
    weight-gradient shape of the AutoVC step on MI355X (tools/gemm_census.py --sweep)."""
    target = _SPLIT_TARGET if target is None else target
    if tiles is None:  # the 128 x 128 output tiles (the halo conv dW kernel passes its 128 x 160 count)
        tiles = math.ceil(M / 128) * math.ceil(N / 128)
    s = int(target / max(tiles, 1) + 0.5)
    return max(1, min(s, K // min_k))


# ------------------------------------------------------------------------- BN
def bn_partial_buffer(M, C, device):
    return torch.empty(math.ceil(M / 128), C, 2, device=device, dtype=torch.float32)


def bn_finalize(partial, M, C, gamma, beta, rmean, rvar, nbt, momentum, eps):
    dev = partial.device
    mean, rstd, scale, shift = (torch.empty(C, device=dev) for _ in range(4))
    L.call("avc_bn_finalize", partial.data_ptr(), M, C, _ptr(gamma), _ptr(beta), _ptr(rmean), _ptr(rvar), _ptr(nbt),
           float(momentum), float(eps), mean.data_ptr(), rstd.data_ptr(), scale.data_ptr(), shift.data_ptr(), stream())
    return mean, rstd, scale, shift


def bn_eval(rmean, rvar, gamma, beta, eps):
    C = rmean.numel()
    dev = rmean.device
    mean, rstd, scale, shift = (torch.empty(C, device=dev) for _ in range(4))
    L.call("avc_bn_eval", rmean.data_ptr(), rvar.data_ptr(), _ptr(gamma), _ptr(beta), C, float(eps), mean.data_ptr(),
           rstd.data_ptr(), scale.data_ptr(), shift.data_ptr(), stream())
    return mean, rstd, scale, shift


def bn_stats(y, M, C, ld=None):
    partial = bn_partial_buffer(M, C, y.device)
    L.call("avc_bn_stats", y.data_ptr(), int(C if ld is None else ld), M, C, partial.data_ptr(), stream())
    return partial


def _twin_buf(t, want):
    """bf16 twin buffer for an fp32 activation in bf16 compute mode (GEMM operand copy)."""
    if want is None:
        want = _COMPUTE == BF16
    return torch.empty(t.shape, device=t.device, dtype=torch.bfloat16) if want else None


def attach_twin(t, t16):
    """Record t16 (bf16, same layout) as the GEMM-operand twin of fp32 t: operand() uses it
    in bf16 compute mode (the bf16 products are identical; the loads are half as wide)."""
    if t16 is not None:
        t._bf16 = t16
    return t


def twin(t):
    """The bf16 twin of t, made by one conversion pass if t has none (bf16 mode only)."""
    if _COMPUTE != BF16 or t.dtype != torch.float32:
        return t
    tw = getattr(t, "_bf16", None)
    if tw is None:
        tw = convert(t.contiguous(), BF16)
        t._bf16 = tw
    return t


def bn_apply(y, scale, shift, act, residual=None, out=None, twin16=None, out_bf16=False):
    """act(y*scale + shift) (+ residual); y fp32 or bf16.  out_bf16: the result is a bf16 tensor
    (no fp32 copy -- an inter-layer activation only ever read as a bf16 GEMM operand); otherwise
    fp32 with a bf16 twin in bf16 compute mode."""
    M, C = y.shape
    if out_bf16:
        o16 = torch.empty(M, C, device=y.device, dtype=torch.bfloat16)
        L.call("avc_bn_apply", y.data_ptr(), _dt(y), scale.data_ptr(), shift.data_ptr(), _ptr(residual), None,
               o16.data_ptr(), M, C, int(act), stream())
        return o16
    out = torch.empty(M, C, device=y.device) if out is None else out
    o16 = _twin_buf(out, twin16)
    L.call("avc_bn_apply", y.data_ptr(), _dt(y), scale.data_ptr(), shift.data_ptr(), _ptr(residual), out.data_ptr(),
           _ptr(o16), M, C, int(act), stream())
    return attach_twin(out, o16)


def bn_bwd(dA, a, y, mean, rstd, gamma, act, need_dbias=True, into=None, twin16=None, beta=None, dy_bf16=False):
    """into = (dgamma, dbeta, dbias) buffers to accumulate into (direct gradient sink).
    a = None: the activation derivative comes from the pre-activation (y-mean)*rstd*gamma + beta.
    dA and y may be fp32 or bf16; dy_bf16: dy is returned as a bf16 tensor only (it feeds bf16
    GEMMs alone), else fp32 with a bf16 twin in bf16 compute mode."""
    M, C = y.shape
    dev = y.device
    if dy_bf16:
        dy, d16 = None, torch.empty(M, C, device=dev, dtype=torch.bfloat16)
    else:
        dy = torch.empty(M, C, device=dev)
        d16 = _twin_buf(dy, twin16)
    if into is not None:
        dgamma, dbeta, dbias = into
    else:
        dgamma = torch.empty(C, device=dev)
        dbeta = torch.empty(C, device=dev)
        dbias = torch.empty(C, device=dev) if need_dbias else None
    ws = torch.empty(int(L.lib().avc_bn_bwd_ws(M, C)), device=dev)
    L.call("avc_bn_bwd", dA.data_ptr(), _dt(dA), _ptr(a), y.data_ptr(), _dt(y), mean.data_ptr(), rstd.data_ptr(),
           _ptr(gamma), _ptr(beta), M, C, int(act), _ptr(dy), _ptr(d16), _ptr(dgamma), _ptr(dbeta), _ptr(dbias),
           int(into is not None), ws.data_ptr(), stream())
    out = d16 if dy_bf16 else attach_twin(dy, d16)
    return out, dgamma, dbeta, dbias


def bn_bwd_apply(dA, y, coef, act, dy_bf16=False, twin16=None):
    """The apply half of the BN backward with avc_gemm_bnb's constants (see bn_bwd)."""
    M, C = y.shape
    dev = y.device
    if dy_bf16:
        dy, d16 = None, torch.empty(M, C, device=dev, dtype=torch.bfloat16)
    else:
        dy = torch.empty(M, C, device=dev)
        d16 = _twin_buf(dy, twin16)
    L.call("avc_bn_bwd_apply", dA.data_ptr(), _dt(dA), y.data_ptr(), _dt(y), coef.data_ptr(), M, C, int(act),
           _ptr(dy), _ptr(d16), stream())
    return d16 if dy_bf16 else attach_twin(dy, d16)


def colsum(x, M, N, ld=None, out=None, accumulate=False, out2=None):
    """Column sums of an (M, N) block (rows ld apart) into out (and the same into out2)."""
    dev = x.device
    out = torch.empty(N, device=dev) if out is None else out
    ws = torch.empty(int(L.lib().avc_colsum_ws(M, N)), device=dev)
    L.call("avc_colsum", x.data_ptr(), int(N if ld is None else ld), M, N, out.data_ptr(), _ptr(out2),
           int(accumulate), ws.data_ptr(), stream())
    return out


# ------------------------------------------------------------------------- LSTM
def lstm_scratch(B, H, dirs, device):
    """bf16 scratch for the large-H recurrence: per-step ping-pong h (2*dirs*B*H bf16) or,
    for the persistent kernel, control words + per-member flags (< 8 KB) + a [2][B][H] payload
    of bf16 (flag form) or of 8-byte {2 x bf16, tag} granules (granule form: 8*B*H bytes)."""
    return torch.zeros(max(2 * dirs * B * H, 4 * B * H + 4096), device=device, dtype=torch.bfloat16)


def lstm_timeout_flag(hbuf, B, H):
    return int(hbuf.view(torch.int32)[0].item())


def lstm_persistent_fwd(B, H, dirs):
    """Whether avc_lstm_fwd takes the one-launch persistent path (asked of lstm.hip: shape,
    compute mode and the occupancy check of the whole grid)."""
    return bool(L.lib().avc_lstm_persistent(int(B), int(H), int(dirs), _COMPUTE, 0))


# ------------------------------------------------------------------------- fault word
_FAULT = {}


def fault_word(device=None):
    """The per-device u32 fault word registered with the library (avc_set_fault_word): bit 0
    = a persistent LSTM recurrence timed out its bounded spin and left its outputs unfinished.
    Created (zeroed) and registered on first use; every persistent launch reports into it."""
    idx = None if device is None else torch.device(device).index
    dev = torch.device("cuda", torch.cuda.current_device() if idx is None else idx)
    w = _FAULT.get(dev.index)
    if w is None:
        with torch.cuda.device(dev):
            w = torch.zeros(1, device=dev, dtype=torch.int32)
            L.call("avc_set_fault_word", w.data_ptr())
        _FAULT[dev.index] = w
    return w


class DeviceFault(RuntimeError):
    """A HIP kernel reported a failure through the fault word (see fault_word)."""


FAULT_BITS = {1: "persistent LSTM recurrence spin timeout (a workgroup of the grid was not resident or stalled; "
                 "the step's outputs are invalid)",
              2: "fused BatchNorm apply: column-tile barrier timeout in a halo conv epilogue (the step's outputs "
                 "are invalid)"}


def raise_on_fault(value):
    v = int(value)
    if v:
        what = "; ".join(msg for bit, msg in FAULT_BITS.items() if v & bit) or "unknown fault bits"
        raise DeviceFault(f"autoformer_amd device fault word = {v:#x}: {what}")


def check_faults(device=None):
    """Synchronous check of the fault word (reads it back; raises DeviceFault if set)."""
    raise_on_fault(fault_word(device).item())


def clear_faults(device=None):
    fault_word(device).zero_()


def lstm_set_spin(spins: int) -> None:
    """Debug: spin bound of the persistent recurrences (0 restores the default; -1 injects a
    timeout at every wait, deterministically)."""
    L.call("avc_lstm_set_spin", int(spins) & 0xFFFFFFFF)


# ---------------------------------------------------------------- collective / recurrence ordering
# A persistent recurrence (lstm_persist_* / lstm2_persist_*: every workgroup of the grid spins on flags
# the others publish) needs its whole grid resident.  RCCL's kernels are polling waves that
# hold CU slots until the peer ranks arrive, so a recurrence launched while a collective is resident
# can wait on workgroups that cannot be scheduled (round 5 measured the same hazard with device-side
# waits: `persistent LSTM recurrence spin timeout`, profiles/r5_graph_modes.txt).  The training step
# keeps them apart by stream order: a collective is enqueued on the comm stream only after
# the decoder recurrences' backward, and the main stream joins the comm stream before the next
# recurrence.  TrainStep reports both points here, and every launch site of a decoder (H > 64)
# recurrence asserts the invariant on the host -- in eager steps and while a step is recorded, so a
# recorded replay inherits it.
_OUTSTANDING = []  # collectives enqueued on another stream and not yet joined by the main stream
_ORDER_STATS = {"checks": 0, "enqueued": 0}  # tests: the invariant was exercised


def collective_enqueued(what: str) -> None:
    _OUTSTANDING.append(what)
    _ORDER_STATS["enqueued"] += 1


def ordering_stats():
    return dict(_ORDER_STATS)


def collective_joined() -> None:
    _OUTSTANDING.clear()


def collectives_outstanding():
    return list(_OUTSTANDING)


def _assert_no_collective(what: str) -> None:
    _ORDER_STATS["checks"] += 1
    if _OUTSTANDING:
        raise RuntimeError(f"{what}: a persistent recurrence was enqueued while the collective(s) {_OUTSTANDING} "
                           "are outstanding on the comm stream; its grid could wait on CU slots held by RCCL's "
                           "polling kernels (DESIGN §6: join the comm stream first)")


def lstm_fwd(xproj, w_hh, B, T, H, dirs, hbuf=None):
    if H > 64:
        _assert_no_collective("avc_lstm_fwd")
    dev = xproj.device
    h = torch.empty(B * T, dirs * H, device=dev)
    c = torch.empty(B * T, dirs * H, device=dev)
    g = torch.empty(B * T, dirs * 4 * H, device=dev)
    h16 = None
    if H > 64:
        fault_word(dev)
    # the bf16 twin of h (the next GEMMs' operand) comes out of the recurrence itself: always on
    # the small-H path in bf16 mode, and on the persistent large-H path
    if (H <= 64 and _COMPUTE == BF16) or (hbuf is not None and H > 64 and lstm_persistent_fwd(B, H, dirs)):
        h16 = torch.empty(B * T, dirs * H, device=dev, dtype=torch.bfloat16)
    L.call("avc_lstm_fwd", xproj.data_ptr(), w_hh.data_ptr(), _dt(w_hh), B, T, H, dirs, h.data_ptr(), _ptr(h16),
           c.data_ptr(), g.data_ptr(), _ptr(hbuf), _COMPUTE, stream())
    return attach_twin(h, h16), c, g


def lstm2_persistent(B, H, in1):
    """Whether avc_lstm2_fwd (two stacked layers, one wavefront launch) applies to this shape."""
    return bool(L.lib().avc_lstm2_persistent(int(B), int(H), int(in1), _COMPUTE))


def lstm2_fwd(xproj0, w_hh0, w_ih1, w_hh1, bias1, B, T, H):
    """Forward of two stacked unidirectional layers in one persistent launch (layer wavefront).
    Returns (h0, c0, gates0, h1, c1, gates1); h0/h1 carry their bf16 twins."""
    _assert_no_collective("avc_lstm2_fwd")
    dev = xproj0.device
    fault_word(dev)
    outs = []
    for _ in range(2):
        outs += [torch.empty(B * T, H, device=dev), torch.empty(B * T, H, device=dev, dtype=torch.bfloat16),
                 torch.empty(B * T, H, device=dev), torch.empty(B * T, 4 * H, device=dev)]
    # zeroed by a fill KERNEL on this stream as well as by the library's memset of the flag words:
    # replayed inside a hipGraph after eager work, the memset node alone left stale flags visible
    # to the wavefront (second replay read the previous replay's payload; tools/graph_fwd_probe.py)
    buf = torch.zeros(int(L.lib().avc_lstm2_scratch_bytes(int(B), int(H))), device=dev, dtype=torch.uint8)
    L.call("avc_lstm2_fwd", xproj0.data_ptr(), w_hh0.data_ptr(), w_ih1.data_ptr(), w_hh1.data_ptr(),
           bias1.data_ptr(), B, T, H, *[o.data_ptr() for o in outs], buf.data_ptr(), stream())
    h0, h0b, c0, g0, h1, h1b, c1, g1 = outs
    _CACHE["lstm2_buf"] = buf  # diagnostics (timeout flag at byte 0); kept alive until the next call
    return attach_twin(h0, h0b), c0, g0, attach_twin(h1, h1b), c1, g1


def lstm2_bwd_persistent(B, H):
    """Whether avc_lstm2_bwd (both lstm2 layers' backward in one wavefront launch) applies."""
    return bool(L.lib().avc_lstm2_bwd_persistent(int(B), int(H), _COMPUTE))


def lstm2_bwd(dh1, c0, g0, c1, g1, wt0, wti1, wt1, B, T, H, fp32=True, db=False):
    """Backward of the two stacked layers in one persistent launch: (dG0, dG1), each fp32 with its
    bf16 twin, or (fp32=False) the bf16 tensors alone.  wt0 / wti1 / wt1: W_hh0^T, W_ih1^T, W_hh1^T
    as bf16 [H][4H].  db: also return the (2, ceil(B/16), 4H) per-group sums of dG over utterances
    and steps (avc_lstm2_bwd db_part), whose column sums are the layers' bias gradients."""
    _assert_no_collective("avc_lstm2_bwd")
    dev = dh1.device
    fault_word(dev)
    outs = [torch.empty(B * T, 4 * H, device=dev) for _ in range(2)] if fp32 else [None, None]
    o16 = [torch.empty(B * T, 4 * H, device=dev, dtype=torch.bfloat16) for _ in range(2)]
    dbp = torch.empty(2, -(-B // 16), 4 * H, device=dev) if db else None
    buf = torch.empty(int(L.lib().avc_lstm2_bwd_scratch_bytes(int(B), int(H))), device=dev, dtype=torch.uint8)
    timed = LAUNCH_TIMING is not None and H == LAUNCH_TIMING_H
    if timed:
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
    rec = L._REC if H == LAUNCH_TIMING_H else None
    if rec is not None:
        box, s = [], torch.cuda.current_stream()
        rec.add_marker(lambda: _timing_mark(box, s, 0))
    L.call("avc_lstm2_bwd", dh1.data_ptr(), c0.data_ptr(), g0.data_ptr(), c1.data_ptr(), g1.data_ptr(), wt0.data_ptr(),
           wti1.data_ptr(), wt1.data_ptr(), B, T, H, _ptr(outs[0]), o16[0].data_ptr(), _ptr(outs[1]),
           o16[1].data_ptr(), buf.data_ptr(), _ptr(dbp), stream())
    if rec is not None:
        rec.add_marker(lambda: _timing_mark(box, s, 1))
    if timed:
        ev[1].record()
        LAUNCH_TIMING.append(ev)
    _CACHE["lstm2_bwd_buf"] = buf  # kept alive until the next call (the launch is asynchronous)
    dg = (attach_twin(outs[0], o16[0]), attach_twin(outs[1], o16[1])) if fp32 else (o16[0], o16[1])
    return (*dg, dbp) if db else dg


def lstm_persistent_bwd(B, H, dirs):
    """Whether avc_lstm_bwd takes the one-launch persistent path (asked of lstm.hip)."""
    return bool(L.lib().avc_lstm_persistent(int(B), int(H), int(dirs), _COMPUTE, 1))


def num_cus():
    if "cus" not in _CACHE:
        _CACHE["cus"] = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    return _CACHE["cus"]


_CACHE = {}


def lstm_bwd_scratch(B, H, dirs, device):
    nbytes = int(L.lib().avc_lstm_bwd_scratch_bytes(int(B), int(H), int(dirs)))
    return torch.empty((nbytes + 1) // 2, device=device, dtype=torch.bfloat16)


def lstm_bwd_timeout_flag(gbuf, B, H):
    return int(gbuf.view(torch.int32)[0].item())


# Diagnostics for bench.py's roofline: when this is a list, every persistent backward
# recurrence launch with H == LAUNCH_TIMING_H appends a (start, end) HIP event pair recorded
# on the launch stream around it (no synchronisation; read after the timed region).
LAUNCH_TIMING = None
LAUNCH_TIMING_H = 1024


def lstm_bwd(dh, h, c, g, w_hh, w_hh_t, B, T, H, dirs, gbuf=None):
    """dL/d(pre-activation gates); in the persistent bf16 mode also its bf16 twin."""
    if H > 64:
        _assert_no_collective("avc_lstm_bwd")
    dev = dh.device
    dg = torch.empty(B * T, dirs * 4 * H, device=dev)
    dcbuf = dg16 = None
    wdt = _dt(w_hh if w_hh_t is None else w_hh_t)
    if H > 64:
        fault_word(dev)
        dcbuf = torch.empty(dirs * B * H, device=dev)
        if _COMPUTE == BF16:
            if gbuf is None:
                gbuf = lstm_bwd_scratch(B, H, dirs, dev)
            if lstm_persistent_bwd(B, H, dirs):
                dg16 = torch.empty(B * T, 4 * H, device=dev, dtype=torch.bfloat16)
    elif _COMPUTE == BF16:
        dg16 = torch.empty(B * T, dirs * 4 * H, device=dev, dtype=torch.bfloat16)
    timed = LAUNCH_TIMING is not None and dg16 is not None and H == LAUNCH_TIMING_H
    if timed:
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
    rec = L._REC if dg16 is not None and H == LAUNCH_TIMING_H else None
    if rec is not None:  # a recorded step (replay.py) times this launch whenever LAUNCH_TIMING is on at replay
        box, s = [], torch.cuda.current_stream()
        rec.add_marker(lambda: _timing_mark(box, s, 0))
    L.call("avc_lstm_bwd", dh.data_ptr(), h.data_ptr(), c.data_ptr(), g.data_ptr(), _ptr(w_hh), _ptr(w_hh_t), wdt, B,
           T, H, dirs, dg.data_ptr(), _ptr(dg16), _ptr(dcbuf), _ptr(gbuf), _COMPUTE, stream())
    if rec is not None:
        rec.add_marker(lambda: _timing_mark(box, s, 1))
    if timed:
        ev[1].record()
        LAUNCH_TIMING.append(ev)
    return attach_twin(dg, dg16)


def _timing_mark(box, s, end):
    if LAUNCH_TIMING is None:
        return
    if not end:
        box[:] = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))]
        box[0][0].record(s)
    elif box:
        box[0][1].record(s)
        LAUNCH_TIMING.append(box.pop())


# ------------------------------------------------------------------------- glue
def enc_concat(mel2d, emb, B, T):
    nm, de = mel2d.shape[1], emb.shape[1]
    out = torch.empty(B * T, nm + de, device=mel2d.device)
    L.call("avc_enc_concat", mel2d.data_ptr(), nm, emb.data_ptr(), out.data_ptr(), B, T, nm, de, stream())
    return out


def codes_gather(lo, B, T, D, freq):
    codes = torch.empty(B, (T // freq) * 2 * D, device=lo.device)
    L.call("avc_codes_gather", lo.data_ptr(), codes.data_ptr(), B, T, D, freq, stream())
    return codes


def codes_scatter(dcodes, B, T, D, freq):
    dlo = torch.empty(B * T, 2 * D, device=dcodes.device)
    L.call("avc_codes_scatter", dcodes.data_ptr(), dlo.data_ptr(), B, T, D, freq, stream())
    return dlo


def dec_concat(codes, emb, B, T, nc, cd):
    de = emb.shape[1]
    out = torch.empty(B * T, cd + de, device=codes.device)
    L.call("avc_dec_concat", codes.data_ptr(), emb.data_ptr(), out.data_ptr(), B, T, nc, cd, de, stream())
    return out


def expand_codes(pc, pe, B, T, nc):
    """(B*T, G) rows pc[b*nc + t // (T/nc)] + pe[b] (lstm1 input projection folded per code)."""
    _dev(pc, pe)
    G = pc.shape[1]
    out = torch.empty(B * T, G, device=pc.device)
    L.call("avc_expand_codes", pc.data_ptr(), pe.data_ptr(), out.data_ptr(), B, T, nc, G, stream())
    return out


def code_cat(codes, emb, B, nc, cd):
    """(B*nc, cd+de) bf16 rows [code_j ; emb_b]: the folded lstm1's GEMM operand (avc_code_cat)."""
    _dev(codes, emb)
    de = emb.shape[1]
    out = torch.empty(B * nc, cd + de, device=codes.device, dtype=torch.bfloat16)
    L.call("avc_code_cat", codes.data_ptr(), emb.data_ptr(), out.data_ptr(), B, nc, cd, de, stream())
    return out


def lstm_fwd_fold(pcode, nc, w_hh, B, T, H, hbuf):
    """Persistent lstm1 forward reading step t's input projection from pcode[b*nc + t // (T/nc)]
    (avc_lstm_fwd_fold); returns h (bf16 twin attached), c, gates as lstm_fwd."""
    _assert_no_collective("avc_lstm_fwd_fold")
    dev = pcode.device
    fault_word(dev)
    h = torch.empty(B * T, H, device=dev)
    h16 = torch.empty(B * T, H, device=dev, dtype=torch.bfloat16)
    c = torch.empty(B * T, H, device=dev)
    g = torch.empty(B * T, 4 * H, device=dev)
    L.call("avc_lstm_fwd_fold", pcode.data_ptr(), nc, w_hh.data_ptr(), B, T, H, h.data_ptr(), h16.data_ptr(),
           c.data_ptr(), g.data_ptr(), hbuf.data_ptr(), stream())
    return attach_twin(h, h16), c, g


def lstm_bwd_fold(dh, c, g, w_hh_t, B, T, H, nc, gbuf=None):
    """Persistent lstm1 backward (avc_lstm_bwd_fold): dG as bf16 only, and s_code (B*nc, 4H) =
    dG summed over each code's frames (fp32, bf16 twin attached)."""
    _assert_no_collective("avc_lstm_bwd_fold")
    dev = dh.device
    fault_word(dev)
    if gbuf is None:
        gbuf = lstm_bwd_scratch(B, H, 1, dev)
    dg16 = torch.empty(B * T, 4 * H, device=dev, dtype=torch.bfloat16)
    sc = torch.empty(B * nc, 4 * H, device=dev)
    sc16 = torch.empty(B * nc, 4 * H, device=dev, dtype=torch.bfloat16)
    L.call("avc_lstm_bwd_fold", dh.data_ptr(), c.data_ptr(), g.data_ptr(), w_hh_t.data_ptr(), B, T, H, nc, None,
           dg16.data_ptr(), sc.data_ptr(), sc16.data_ptr(), gbuf.data_ptr(), stream())
    return dg16, attach_twin(sc, sc16)


def dec_concat_bwd(dout, B, T, nc, cd, de):
    dcodes = torch.empty(B, nc * cd, device=dout.device)
    L.call("avc_dec_concat_bwd", dout.data_ptr(), dcodes.data_ptr(), B, T, nc, cd, de, stream())
    return dcodes


# ------------------------------------------------------------------------- weights
def conv_pack(w, mode, dtype):
    Co, Ci, K = w.shape
    tdt = torch.bfloat16 if dtype == BF16 else torch.float32
    out = torch.empty(Co * Ci * K, device=w.device, dtype=tdt)
    L.call("avc_conv_pack", w.data_ptr(), out.data_ptr(), dtype, Co, Ci, K, int(mode), stream())
    return out.view(Co, K * Ci) if mode == 0 else out.view(Ci, K * Co)


def conv_pack_slice(w, ci0, cn, cpad, mode, dtype):
    """Pack input channels [ci0, ci0+cn) of conv weight w (Co, Ci, K), channel axis zero-padded to
    cpad: mode 0 -> (Co, K*cpad), 1 -> (cpad, K*Co) (flipped taps), 2 -> (K*Co, cpad); mode 3 pads
    the OUTPUT channel axis instead: (cn, K*cpad), flipped taps, cpad >= Co (a data-gradient pack
    whose dy operand has cpad columns)."""
    Co, Ci, Kw = w.shape
    tdt = torch.bfloat16 if dtype == BF16 else torch.float32
    out = torch.empty((cn if mode == 3 else Co) * cpad * Kw, device=w.device, dtype=tdt)
    L.call("avc_conv_pack_slice", w.data_ptr(), out.data_ptr(), dtype, Co, Ci, Kw, ci0, cn, cpad, mode, stream())
    if mode == 3:
        return out.view(cn, Kw * cpad)
    return out.view(*((Co, Kw * cpad) if mode == 0 else (cpad, Kw * Co) if mode == 1 else (Kw * Co, cpad)))


def conv_edge_table(E, B, Co, Kw, T, pad):
    """S[b][cls][co]: the sum of E[b][k][co] over the taps valid at each edge class (fold.hip)."""
    _dev(E)
    S = torch.empty(B * (2 * pad + 1), Co, device=E.device)
    L.call("avc_conv_edge_table", E.data_ptr(), B, Co, Kw, T, pad, S.data_ptr(), stream())
    return S


def conv_edge_colsum(dy, B, T, C, Kw, pad):
    """(B*Kw, C): per utterance and tap, the column sums of dy over the frames the tap reads."""
    _dev(dy)
    out = torch.empty(B * Kw, C, device=dy.device)
    L.call("avc_conv_edge_colsum", dy.data_ptr(), _dt(dy), B, T, C, Kw, pad, out.data_ptr(), stream())
    return out


def disc_dense_fwd(a, w, bias, B, nl, nc):
    """Discriminator head: sigmoid(bias + a . w) per utterance with a bin-major [B][nl*nc] and w
    the channel-major dense1.weight (nc*nl).  Returns p (B, 1)."""
    _dev(a)
    p = torch.empty(B, 1, device=a.device)
    L.call("avc_disc_dense_fwd", a.data_ptr(), w.data_ptr(), _ptr(bias), B, nl, nc, None, p.data_ptr(), stream())
    return p


def disc_dense_bwd(dp, p, a, w, B, nl, nc):
    """(da [B][nl*nc], dw (1, nc*nl), dbias (1,)) from dL/dp through the sigmoid."""
    da = torch.empty(B, nl * nc, device=a.device)
    dw = torch.empty(1, nc * nl, device=a.device)
    db = torch.empty(1, device=a.device)
    L.call("avc_disc_dense_bwd", dp.data_ptr(), p.data_ptr(), a.data_ptr(), w.data_ptr(), B, nl, nc, da.data_ptr(),
           dw.data_ptr(), db.data_ptr(), stream())
    return da, dw, db


def conv_grad_unpack_slice(dwf, ld, kstride, dw, ci0, cn, accumulate=True):
    """dw[co][ci0+ci][k] (+)= dwf[co*ld + k*kstride + ci], ci < cn."""
    Co, Ci, Kw = dw.shape
    L.call("avc_conv_grad_unpack_slice", dwf.data_ptr(), int(ld), int(kstride), dw.data_ptr(), Co, Ci, Kw, ci0, cn,
           int(accumulate), stream())
    return dw


def conv_grad_unpack(dwf, Co, Ci, K, into=None):
    dw = torch.empty(Co, Ci, K, device=dwf.device) if into is None else into
    L.call("avc_conv_grad_unpack", dwf.data_ptr(), dw.data_ptr(), Co, Ci, K, int(into is not None), stream())
    return dw


def convert(src, dtype, out=None):
    tdt = torch.bfloat16 if dtype == BF16 else torch.float32
    out = torch.empty(src.shape, device=src.device, dtype=tdt) if out is None else out
    L.call("avc_convert", src.data_ptr(), out.data_ptr(), dtype, src.numel(), stream())
    return out


def transpose(src, dtype, out=None, ld_out=0):
    """out[c][r] = src[r][c] (out rows ld_out apart: a column block of a wider matrix)."""
    R, C = src.shape
    tdt = torch.bfloat16 if dtype == BF16 else torch.float32
    out = torch.empty(C, R, device=src.device, dtype=tdt) if out is None else out
    L.call("avc_transpose", src.data_ptr(), out.data_ptr(), dtype, R, C, int(ld_out), stream())
    return out


def add(a, b, out=None):
    out = torch.empty_like(a) if out is None else out
    L.call("avc_add", a.data_ptr(), b.data_ptr(), out.data_ptr(), a.numel(), stream())
    return out


# ------------------------------------------------------------------------- losses / optimizer
def mse_loss(a, b):
    out = torch.empty((), device=a.device)
    L.call("avc_mse_loss", a.data_ptr(), b.data_ptr(), a.numel(), out.data_ptr(), stream())
    return out


def l1_loss(a, b):
    out = torch.empty((), device=a.device)
    L.call("avc_l1_loss", a.data_ptr(), b.data_ptr(), a.numel(), out.data_ptr(), stream())
    return out


def loss_grad(a, b, dloss, mode, sign):
    g = torch.empty_like(a)
    L.call("avc_loss_grad", a.data_ptr(), b.data_ptr(), a.numel(), dloss.data_ptr(), int(mode), g.data_ptr(),
           float(sign), stream())
    return g


def vc_loss(x, y1, y2, ca, cb, lambda_cd):
    """The loss block of Solver.train in one launch (avc_vc_loss): a (4,) device tensor
    [mse(x, y1), mse(x, y2), l1(ca, cb), total]."""
    out = torch.empty(4, device=x.device)
    ws = torch.empty(int(L.lib().avc_vc_loss_ws()), device=x.device)
    L.call("avc_vc_loss", x.data_ptr(), y1.data_ptr(), y2.data_ptr(), x.numel(), ca.data_ptr(), cb.data_ptr(),
           ca.numel(), float(lambda_cd), out.data_ptr(), ws.data_ptr(), stream())
    return out


def vc_loss_grad(x, y1, y2, ca, cb, lambda_cd, d, need):
    """Gradients of vc_loss's outputs (avc_vc_loss_grad): d = 4 upstream device scalars (or
    None), need = (y1, y2, ca, cb) flags; returns the four gradients (None where not needed)."""
    outs = [torch.empty_like(t) if nd else None for t, nd in zip((y1, y2, ca, cb), need)]
    L.call("avc_vc_loss_grad", x.data_ptr(), y1.data_ptr(), y2.data_ptr(), x.numel(), ca.data_ptr(), cb.data_ptr(),
           ca.numel(), float(lambda_cd), *[_ptr(t) for t in d], *[_ptr(t) for t in outs], stream())
    return outs


def adam(p, g, m, v, lr, beta1, beta2, eps, state, advance=True, max_blocks=0):
    L.call("avc_adam_blocks", p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(), float(lr),
           float(beta1), float(beta2), float(eps), state.data_ptr(), int(advance), int(max_blocks), stream())


def act_fwd(x, act, out=None):
    out = torch.empty_like(x) if out is None else out
    L.call("avc_act_fwd", x.data_ptr(), out.data_ptr(), x.numel(), int(act), stream())
    return out


def act_bwd(g, yout, act):
    dx = torch.empty_like(g)
    L.call("avc_act_bwd", g.data_ptr(), yout.data_ptr(), dx.data_ptr(), g.numel(), int(act), stream())
    return dx


def bce_loss(p, target):
    out = torch.empty((), device=p.device)
    L.call("avc_bce_loss", p.data_ptr(), p.numel(), float(target), out.data_ptr(), stream())
    return out


def bce_grad(p, target, dloss, through_sigmoid=False):
    g = torch.empty_like(p)
    L.call("avc_bce_grad", p.data_ptr(), p.numel(), float(target), dloss.data_ptr(), g.data_ptr(),
           int(through_sigmoid), stream())
    return g


# ------------------------------------------------------------------------- MetaFormer blocks
def _ws(rows, C, dev):
    return torch.empty(int(L.lib().avc_norm_ws(rows, C)), device=dev)


def group_norm_fwd(x, B, C, gamma, beta, eps, twin=False):
    """twin (C % 4 == 0): the bf16 operand twin of y written in the same pass."""
    S = x.numel() // B
    y = torch.empty_like(x)
    y16 = _twin_buf(y, None) if twin else None
    mean, rstd = torch.empty(B, device=x.device), torch.empty(B, device=x.device)
    L.call("avc_group_norm_fwd2", x.data_ptr(), B, S, C, _ptr(gamma), _ptr(beta), float(eps), y.data_ptr(), _ptr(y16),
           mean.data_ptr(), rstd.data_ptr(), _ws(x.numel() // C, C, x.device).data_ptr(), stream())
    return (attach_twin(y, y16) if y16 is not None else y), mean, rstd


def group_norm_bwd(dy, x, gamma, mean, rstd, B, C, dgamma=None, dbeta=None, accumulate=False):
    S = x.numel() // B
    dx = torch.empty_like(x)
    L.call("avc_group_norm_bwd", dy.data_ptr(), x.data_ptr(), _ptr(gamma), mean.data_ptr(), rstd.data_ptr(), B, S, C,
           dx.data_ptr(), _ptr(dgamma), _ptr(dbeta), int(accumulate), _ws(x.numel() // C, C, x.device).data_ptr(),
           stream())
    return dx


def ln_vec(D):
    """Whether the one-pass register-row LayerNorm forms apply (norm.hip ln_*_v_kernel)."""
    return D % 4 == 0 and D <= 512


def layer_norm_fwd(x, gamma, beta, eps, out_bf16=False):
    """out_bf16: y as a bf16 tensor only (an operand read only by bf16 GEMMs / transposes)."""
    R, D = x.shape
    mean, rstd = torch.empty(R, device=x.device), torch.empty(R, device=x.device)
    if out_bf16 and not ln_vec(D):
        # the one-pass bf16 form holds a row in registers (D % 4 == 0, D <= 512): otherwise the
        # fp32 LayerNorm, then a convert pass
        y = torch.empty(R, D, device=x.device)
        L.call("avc_layer_norm_fwd2", x.data_ptr(), R, D, _ptr(gamma), _ptr(beta), float(eps), y.data_ptr(), None,
               mean.data_ptr(), rstd.data_ptr(), stream())
        return convert(y, BF16), mean, rstd
    y = torch.empty(R, D, device=x.device, dtype=torch.bfloat16 if out_bf16 else torch.float32)
    L.call("avc_layer_norm_fwd2", x.data_ptr(), R, D, _ptr(gamma), _ptr(beta), float(eps),
           None if out_bf16 else y.data_ptr(), y.data_ptr() if out_bf16 else None, mean.data_ptr(), rstd.data_ptr(),
           stream())
    return y, mean, rstd


def layer_norm_bwd(dy, x, gamma, mean, rstd, dgamma=None, dbeta=None, accumulate=False, residual=None, twin=False,
                   row_sum=None):
    """dx (+ residual: the gradient of a residual branch around the norm, added in the same pass;
    twin: its bf16 operand twin written beside it; row_sum: a (R,) tensor receiving each row's sum of dx)."""
    R, D = x.shape
    dx = torch.empty_like(x)
    dx16 = _twin_buf(dx, None) if twin else None
    if not ln_vec(D) and (residual is not None or twin or row_sum is not None):
        # the one-pass form (residual add, bf16 twin, row sums in the same pass) needs D % 4 == 0 and
        # D <= 512: otherwise the plain backward, then the add / convert passes
        if row_sum is not None:
            raise RuntimeError("layer_norm_bwd: row sums need D % 4 == 0 and D <= 512")
        L.call("avc_layer_norm_bwd", dy.data_ptr(), x.data_ptr(), _ptr(gamma), mean.data_ptr(), rstd.data_ptr(), R, D,
               dx.data_ptr(), _ptr(dgamma), _ptr(dbeta), int(accumulate), _ws(R, D, x.device).data_ptr(), stream())
        if residual is not None:
            add(dx, residual, out=dx)
        if dx16 is not None:
            convert(dx, BF16, out=dx16)
            return attach_twin(dx, dx16)
        return dx
    L.call("avc_layer_norm_bwd2", dy.data_ptr(), x.data_ptr(), _ptr(gamma), mean.data_ptr(), rstd.data_ptr(), R, D,
           _ptr(residual), dx.data_ptr(), _ptr(dx16), _ptr(row_sum), _ptr(dgamma), _ptr(dbeta), int(accumulate),
           _ws(R, D, x.device).data_ptr(), stream())
    return attach_twin(dx, dx16) if dx16 is not None else dx


def gelu_bwd(g, x):
    dx = torch.empty_like(x)
    L.call("avc_gelu_bwd", g.data_ptr(), x.data_ptr(), dx.data_ptr(), x.numel(), stream())
    return dx


def pool3_mixer(x, B, Lf, C, backward=False):
    y = torch.empty_like(x)
    L.call("avc_pool3_mixer", x.data_ptr(), y.data_ptr(), B, Lf, C, int(backward), stream())
    return y


def patchify(src, B, Lf, C, ps, backward=False, out_bf16=False):
    """out_bf16 (forward only): the patches as a bf16 tensor (a GEMM operand alone)."""
    if out_bf16 and not backward:
        dst = torch.empty(B * (C // ps) * (Lf // ps), ps * ps, device=src.device, dtype=torch.bfloat16)
        L.call("avc_patchify16", src.data_ptr(), dst.data_ptr(), B, Lf, C, int(ps), stream())
        return dst
    if backward:
        dst = torch.empty(B * Lf, C, device=src.device)
    else:
        dst = torch.empty(B * (C // ps) * (Lf // ps), ps * ps, device=src.device)
    L.call("avc_patchify", src.data_ptr(), dst.data_ptr(), B, Lf, C, int(ps), int(backward), stream())
    return dst


def transpose_batched(src, B, R, C, out=None, accumulate=False):
    dst = torch.empty(B * C * R, device=src.device) if out is None else out
    L.call("avc_transpose_batched", src.data_ptr(), dst.data_ptr(), B, R, C, int(accumulate), stream())
    return dst


def transpose_pad(src, B, R, C, ld, dtype=F32, twin=False):
    """(B*C, ld) per-utterance transpose of src (B, R, C), rows zero-padded from R to ld, in dtype;
    twin (fp32 dtype only): the bf16 operand twin written in the same pass (avc_transpose_batched2)."""
    if dtype == BF16:
        out, o16 = None, torch.empty(B * C, ld, device=src.device, dtype=torch.bfloat16)
    else:
        out = torch.empty(B * C, ld, device=src.device)
        o16 = _twin_buf(out, None) if twin else None
    L.call("avc_transpose_batched2", src.data_ptr(), _dt(src), _ptr(out), _ptr(o16), B, R, C, int(ld), 0, stream())
    if dtype == BF16:
        return o16
    return attach_twin(out, o16) if o16 is not None else out


# ------------------------------------------------------------------------- AdaIN / Adjust variants
def moments(x, out=None):
    """[x.mean(), x.std()] (unbiased) of the whole tensor, on device (variants.hip)."""
    _dev(x)
    out = torch.empty(2, device=x.device) if out is None else out
    ws = torch.empty(int(L.lib().avc_moments_ws()), device=x.device, dtype=torch.float64)
    L.call("avc_moments", x.data_ptr(), x.numel(), ws.data_ptr(), out.data_ptr(), stream())
    return out


def moments_bwd(x, mom, dmean, dstd):
    """dx of the two moments; dmean / dstd are device scalars (views) or None."""
    dx = torch.empty_like(x)
    L.call("avc_moments_bwd", x.data_ptr(), x.numel(), mom.data_ptr(), _ptr(dmean), _ptr(dstd), None,
           dx.data_ptr(), stream())
    return dx


def adain_fwd(x, mom, mu, sigma):
    y = torch.empty_like(x)
    L.call("avc_adain_fwd", x.data_ptr(), x.numel(), mom.data_ptr(), mu.data_ptr(), sigma.data_ptr(), y.data_ptr(),
           stream())
    return y


def adain_bwd(g, x, mom, sigma):
    """(dx, dmu, dsigma) of y = (x - mean x) / std x * sigma + mu."""
    dev = x.device
    dx = torch.empty_like(x)
    sums = torch.empty(2, device=dev)
    dmu, dsig = torch.empty((), device=dev), torch.empty((), device=dev)
    ws = torch.empty(int(L.lib().avc_moments_ws()), device=dev, dtype=torch.float64)
    L.call("avc_adain_bwd", g.data_ptr(), x.data_ptr(), x.numel(), mom.data_ptr(), sigma.data_ptr(), ws.data_ptr(),
           sums.data_ptr(), dx.data_ptr(), dmu.data_ptr(), dsig.data_ptr(), stream())
    return dx, dmu, dsig


def segsum(x, B, T, C, ld, out=None, accumulate=False):
    """out (B, C) = per-utterance sum over T of a C-column block of frame-major rows ld apart."""
    _dev(x)
    out = torch.empty(B, C, device=x.device) if out is None else out
    L.call("avc_segsum", x.data_ptr(), int(ld), B, T, C, out.data_ptr(), int(accumulate), stream())
    return out


def step_select(h, B, T, t):
    C = h.shape[1]
    out = torch.empty(B, C, device=h.device)
    L.call("avc_step_select", h.data_ptr(), out.data_ptr(), B, T, t, C, 0, stream())
    return out


def step_scatter(d, B, T, t):
    C = d.shape[1]
    out = torch.empty(B * T, C, device=d.device)
    L.call("avc_step_select", d.data_ptr(), out.data_ptr(), B, T, t, C, 1, stream())
    return out


def rownorm_fwd(x):
    R, C = x.shape
    y = torch.empty_like(x)
    norms = torch.empty(R, device=x.device)
    L.call("avc_rownorm_fwd", x.data_ptr(), R, C, y.data_ptr(), norms.data_ptr(), stream())
    return y, norms


def rownorm_bwd(dy, y, norms):
    R, C = y.shape
    dx = torch.empty_like(y)
    L.call("avc_rownorm_bwd", dy.data_ptr(), y.data_ptr(), norms.data_ptr(), R, C, dx.data_ptr(), stream())
    return dx


def pad_cols(src, Cd, dtype=F32, C=None):
    """(R, Cd) copy of the first C columns of the row-major 2-D src, zero-padded (or cropped)."""
    _dev(src)
    R, lds = src.shape
    C = lds if C is None else C
    tdt = torch.bfloat16 if dtype == BF16 else torch.float32
    out = torch.empty(R, Cd, device=src.device, dtype=tdt)
    L.call("avc_pad_cols", src.data_ptr(), lds, out.data_ptr(), dtype, R, C, Cd, stream())
    return out


def crop_add(src, dst, C=None):
    """dst (R, C) += src[:, :C] (src rows may be longer): a padded product cropped into .grad."""
    R, lds = src.shape
    C = dst.shape[-1] if C is None else C
    L.call("avc_crop_add", src.data_ptr(), lds, dst.data_ptr(), R, C, stream())
    return dst


def gelu_fwd_operand(x):
    """GELU(x) as a GEMM operand: in bf16 mode only the bf16 tensor is written (the fp32
    activation is never read by anything but GEMMs); fp32 mode: the fp32 result."""
    if _COMPUTE != BF16:
        return act_fwd(x, ACT_GELU)
    y16 = torch.empty(x.shape, device=x.device, dtype=torch.bfloat16)
    L.call("avc_gelu_twin", None, x.data_ptr(), None, y16.data_ptr(), x.numel(), 0, stream())
    return y16


def gelu_bwd_twin(g, x):
    """g * GELU'(x) in fp32 with its bf16 twin attached (bf16 mode), one pass."""
    dx = torch.empty_like(x)
    d16 = _twin_buf(dx, None)
    L.call("avc_gelu_twin", g.data_ptr(), x.data_ptr(), dx.data_ptr(), _ptr(d16), x.numel(), 1, stream())
    return attach_twin(dx, d16)
