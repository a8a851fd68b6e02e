"""Autograd functions of the AutoVC training path, each a sequence of HIP kernels.

Activations are frame-major 2-D tensors (B*T, C) — the reference's (B, C, T) conv tensors
transposed once at the model boundary, which for AutoVC is free because its inputs and
outputs are already (B, T, 80) (factory/AutoVC.py:46, 208-209).

Weights stay fp32 ``nn.Parameter``s in the reference layout (state_dict parity); the
kernel-side copies (im2col-ordered conv weights, bf16 casts, transposed W_hh, stacked
bidirectional W_ih, b_ih + b_hh) are rebuilt by HIP kernels whenever a parameter changes
(``param._version``) or the optimizer signals an update (``weights_changed()``), i.e. once
per training step.
"""
from __future__ import annotations

import os
import weakref

import torch

from . import kernels as K
from .kernels import operand

_EPOCH = [0]
# diagnostics only (tools/contention_trace.py): skip the side-stream weight-gradient GEMMs (wrong
# gradients; bench.py refuses it)
_ABLATE_WGRAD = os.environ.get("AVC_ABLATE_WGRAD") == "1"

# ---------------------------------------------------------------- gradient sink / side stream
# In "sink" mode (set by TrainStep) parameter gradients are accumulated by the kernels
# straight into the preallocated p.grad views of the flat gradient buffer, and the
# weight-gradient GEMMs (off the critical path of the backward) run on a side stream that
# overlaps the latency-bound LSTM recurrences on the main stream.  The autograd functions
# then return None for parameters.  join_side() must run before the gradients are read.
_SINK = {"on": False, "side": None, "keep": [], "tail": False, "pend": {}}


def set_grad_sink(on: bool) -> None:
    _SINK["on"] = bool(on)
    if on and _SINK["side"] is None:
        _SINK["side"] = torch.cuda.Stream()


# ---- cheap cross-stream ordering: raw HIP events on raw stream handles (events.hip) and
# torch's current stream switched through its C bindings.  torch.cuda.Event() / .record() /
# current_stream() / torch.cuda.stream() cost 10-15 us of Python each (measured ~1 ms per AutoVC
# step at ~90 uses, tools/host_profile2.py); these cost a ctypes call.
_EV = {"ring": [], "i": 0, "gen": 0, "slot": []}
_EV_RING = 512  # events in flight per step are < 100; a handle is re-recorded 5+ steps later


def _ev_next(stream_raw):
    ring = _EV["ring"]
    if not ring:
        import ctypes

        for _ in range(_EV_RING):
            h = ctypes.c_void_p()
            K.L.call("avc_event_create", ctypes.byref(h))
            ring.append(h.value)
        _EV["slot"] = [0] * len(ring)
    i = _EV["i"]
    _EV["i"] = (i + 1) % len(ring)
    _EV["gen"] += 1
    _EV["slot"][i] = _EV["gen"]
    K.L.call("avc_event_record", ring[i], K.stream() if stream_raw is None else stream_raw)
    return i


def ev_record(stream_raw=None):
    """Record a ring event on the raw stream (default: torch's current stream); returns its handle.
    For waits issued right away (within the same step); a wait that may come much later takes
    ev_token / wait_token, which check that the ring slot was not re-recorded meanwhile."""
    return _EV["ring"][_ev_next(stream_raw)]


def ev_token(stream_raw=None):
    """Record a ring event and return (slot, generation) for a later wait_token."""
    i = _ev_next(stream_raw)
    return (i, _EV["slot"][i])


def stream_wait(stream_raw, ev):
    """The raw stream waits for the event's current record."""
    K.L.call("avc_stream_wait_event", stream_raw, ev)


def wait_token(stream_raw, tok):
    """stream_wait on an ev_token's record; raises if the ring slot has been re-recorded since (the
    dependency would silently move to the newer record -- ADVICE r3)."""
    i, gen = tok
    if _EV["slot"][i] != gen:
        raise RuntimeError(f"event ring slot {i} was re-recorded before its wait (> {_EV_RING} records in between)")
    K.L.call("avc_stream_wait_event", stream_raw, _EV["ring"][i])


_get_cur = torch._C._cuda_getCurrentStream
_set_cur = torch._C._cuda_setStream


def on_stream(stream):
    return _OnStream(stream)


class _OnStream:
    """torch's current stream switched to `stream` (allocations and launches go there) through
    the C bindings -- what torch.cuda.stream(stream) does for a single-device process."""

    __slots__ = ("stream", "prev")

    def __init__(self, stream):
        self.stream = stream

    def __enter__(self):
        self.prev = _get_cur(K._cur_device())
        st = self.stream
        _set_cur(stream_id=st.stream_id, device_index=st.device_index, device_type=st.device_type)
        return self

    def __exit__(self, *exc):
        sid, dev, dt = self.prev
        _set_cur(stream_id=sid, device_index=dev, device_type=dt)
        return False


def sink_on() -> bool:
    return _SINK["on"]


def side_stream():
    """The weight-gradient stream (None before set_grad_sink(True))."""
    return _SINK["side"]


def mark():
    """Event on the current stream (sink mode): a later _Side(after=...) starts from here, so
    the critical-path kernels launched in between (data gradients) are not delayed behind
    the host work of queueing the weight-gradient branch."""
    if not _SINK["on"]:
        return None
    return ev_record()


class _Side:
    """Context: run enclosed kernels on the side stream after everything queued so far on
    the current stream (or after the event `after`); tensors passed to keep() stay alive
    until join_side()."""

    def __init__(self, after=None):
        self.after = after

    def __enter__(self):
        side = _SINK["side"]
        stream_wait(side.cuda_stream, self.after if self.after is not None else ev_record())
        self.ctx = _OnStream(side)
        self.ctx.__enter__()
        return self

    def keep(self, *ts):
        _SINK["keep"].extend(t for t in ts if t is not None)

    def __exit__(self, *exc):
        self.ctx.__exit__(*exc)
        return False


def side_wrote(param) -> None:
    """The side stream has just queued an accumulation into param.grad: remember where, so that a
    later accumulation on the main stream (main_wgrad) waits for it."""
    _SINK["pend"][id(param)] = ev_token(_SINK["side"].cuda_stream)


def main_wgrad(param, last=False) -> bool:
    """Whether this layer's weight gradient runs on the main stream, accumulating into param.grad
    there: in the tail of the backward (set_tail: after the decoder's gradients, only the encoder's
    full pass is left, and the main stream would otherwise wait for the side stream's backlog before
    the optimizer step) when AVC_TAIL_WGRAD_MAIN is on.  The main stream first waits for the side
    stream's last accumulation into the same .grad -- the encoder's convs run in the full pass and in
    the re-pass, the re-pass's weight gradients are side-stream kernels, and two read-modify-writes of
    one .grad on two unordered streams lose updates (round 6: a recorded C2 step's conv0 gradient had
    been 1.1e-3 off the eager one, tests/test_gpu_replay.py).  That accumulation was queued long
    before (the re-pass is the first part of the backward), so the wait costs nothing.  last: the
    layer has no data gradient (the encoder's first conv, the last layer of every backward): on the
    main stream in any case."""
    if not (_SINK["on"] and (last or (_SINK["tail"] and _TAIL_WGRAD_MAIN))):
        return False
    tok = _SINK["pend"].pop(id(param), None)
    if tok is not None:
        wait_token(K.stream(), tok)
    return True


def set_tail(on: bool) -> None:
    """From here to the next join_side() the backward is in its tail (see main_wgrad)."""
    _SINK["tail"] = bool(on)


# the encoder's conv weight gradients in the tail of the backward on the main stream (round 6,
# profiles/r6_tail_wgrad_main.txt); "0": on the side stream like every other weight gradient
_TAIL_WGRAD_MAIN = os.environ.get("AVC_TAIL_WGRAD_MAIN", "1") != "0"


def join_side() -> None:
    _SINK["tail"] = False
    _SINK["pend"].clear()
    side = _SINK["side"]
    if side is not None:
        stream_wait(K.stream(), ev_record(side.cuda_stream))
    _SINK["keep"].clear()


def _grad_of(p):
    if p.grad is None:
        raise RuntimeError("gradient sink mode needs preallocated p.grad (see dist.flatten_params_)")
    return p.grad


def weights_changed() -> None:
    """Call after updating parameters through raw pointers (fused Adam, DDP broadcast)."""
    _EPOCH[0] += 1


_PLAN = []  # every PackCache in first-use order (the next step's prefetch plan)


def _pack_key(params):
    return (_EPOCH[0], K.compute(), tuple((p.data_ptr(), p._version) for p in params))


class PackCache:
    """Derived copy of some parameters (packed / transposed / bf16 weights), rebuilt when
    they change.  prefetch_packs() builds the next step's copies on the side stream right
    after the optimizer step; get() then only orders the current stream after that build."""
    __slots__ = ("key", "val", "pending", "params", "build", "ops", "used", "__weakref__")

    def __init__(self):
        self.used = True  # get() since the last prefetch (a forward-graph replay asks for none of its packs)
        self.key = None
        self.val = None
        self.pending = None
        self.params = None
        self.build = None
        self.ops = None  # optional: val -> list of pack ops rebuilding val in place (batched prefetch)

    def get(self, params, build, ops=None):
        self.used = True
        if ops is not None:
            self.ops = ops
        if _FROZEN[0] and self.ops is not None and self.val is not None:
            # graph capture (TrainStep.capture): the captured step rewrites this pack in place
            # after its optimizer step (repack_in_place), so the forward just reads the buffers
            return self.val
        key = _pack_key(params)
        if key != self.key:
            pend, self.pending = self.pending, None
            if pend is not None and pend[0] == key:
                wait_token(K.stream(), pend[2])
                self.val = pend[1]
            else:
                with torch.no_grad():
                    self.val = build()
            self.key = key
            if self.build is None:
                _PLAN.append(weakref.ref(self))
            self.params, self.build = params, build
        return self.val


_FROZEN = [False]  # set while a step is captured: packs with in-place ops are not rebuilt by get()


def freeze_packs(on: bool) -> None:
    _FROZEN[0] = bool(on)
    if on:
        for ref in _PLAN:
            c = ref()
            if c is not None:
                c.pending = None  # a prefetched copy would replace val; the frozen val is rewritten instead


def plan_caches(pred=None):
    """Live caches of the prefetch plan (first-use order) with a built value, filtered by pred."""
    out = []
    for ref in _PLAN:
        c = ref()
        if c is not None and c.val is not None and (pred is None or pred(c)):
            out.append(c)
    return out


def repack_in_place(caches, group):
    """Rewrite the packs of `caches` in place on the current stream from the current parameters:
    one batched avc_pack_batch launch over the caches that describe their packs (PackCache.ops);
    the others are rebuilt (new tensors, get() rebuilds them inline, they are not frozen).  A
    captured step calls this after its optimizer step, so the next replay's forward reads packs of
    the updated weights with no pack kernels of its own (~55 small launches, ~0.35 ms of the C2
    main stream, in one).  The op table is made on the first (eager) call: call it once outside
    the capture with the same `group` first."""
    batched = [c for c in caches if c.ops is not None]
    # one launch per <= _PACK_MAX_OPS ops (the kernel keeps its op table in LDS)
    chunks, cur, n = [], [], 0
    for c in batched:
        k = len(c.ops(c.val))
        if cur and n + k > _PACK_MAX_OPS:
            chunks.append(cur)
            cur, n = [], 0
        cur.append(c)
        n += k
    if cur:
        chunks.append(cur)
    for i, chunk in enumerate(chunks):
        plan = _batch_plan(chunk, (group, i))
        K.L.call("avc_pack_batch", plan["ops"].data_ptr(), plan["prefix"].data_ptr(), plan["n"], plan["total"],
                 K.stream())


_PACK_MAX_OPS = 128  # PACK_MAX_OPS of pack_batch_kernel (elem.hip)


_BATCH = {}       # group index -> device op table of that group of packs


def _op_struct(o):
    from ._lib import PackOp

    st = PackOp()
    st.src = o["src"]
    st.src2 = o.get("src2") or None
    st.dst = o["dst"]
    st.kind = o["kind"]
    st.out_dtype = o["dtype"]
    d = list(o["dims"]) + [0, 0, 0]
    st.d0, st.d1, st.d2 = d[0], d[1], d[2]
    st.ld_out = o.get("ld", 0)
    if "slice" in o:  # CONV_SLICE: (ci0, cn, cpad, mode)
        st.ci0, st.cn, st.cpad, st.mode = o["slice"]
    return st


def _op_len(o):
    """Units of an op in avc_pack_batch (elem.hip pack_batch_kernel): a 64 x 64 transpose tile; an LDS-staged
    conv tile (Wf: 4 output x 64 input channels for <= 16 taps, Wd: 32 x 16 for <= 8 taps); else 4096
    elements (of the destination for a conv0-fold channel slice)."""
    from ._lib import PACK_CONV_D, PACK_CONV_F, PACK_CONV_SLICE, PACK_TRANSPOSE

    d = o["dims"]
    if o["kind"] == PACK_CONV_SLICE:
        _, cn, cpad, mode = o["slice"]
        return -(-((cn if mode == 3 else d[0]) * cpad * d[2]) // 4096)
    if o["kind"] == PACK_TRANSPOSE:
        return -(-d[0] // 64) * -(-d[1] // 64)
    if o["kind"] == PACK_CONV_F and d[2] <= 16:
        return -(-d[0] // 4) * -(-d[1] // 64)
    if o["kind"] == PACK_CONV_D and d[2] <= 8:
        return -(-d[0] // 32) * -(-d[1] // 16)
    n = d[0] * d[1] * d[2] if o["kind"] in (PACK_CONV_F, PACK_CONV_D) else d[0]
    return -(-n // 4096)


def _batch_plan(caches, group=0):
    """Device op table (avc_pack_op[]) + unit prefix for the caches that describe their packs;
    rebuilt only when a cache's buffers or parameters moved."""
    import ctypes

    sig = tuple((id(c), tuple(p.data_ptr() for p in c.params),
                 tuple(t.data_ptr() for t in c.val if t is not None) if isinstance(c.val, tuple) else c.val.data_ptr())
                for c in caches)
    plan = _BATCH.get(group)
    if plan is not None and plan["sig"] == sig:
        return plan
    ops = [o for c in caches for o in c.ops(c.val)]
    arr = (_op_struct_type() * len(ops))(*[_op_struct(o) for o in ops])
    prefix = [0]
    for o in ops:
        prefix.append(prefix[-1] + _op_len(o))
    dev = caches[0].params[0].device
    raw = torch.frombuffer(bytearray(ctypes.string_at(ctypes.addressof(arr), ctypes.sizeof(arr))), dtype=torch.uint8)
    plan = {"sig": sig, "ops": raw.to(dev), "prefix": torch.tensor(prefix, dtype=torch.int64).to(dev), "n": len(ops),
            "total": prefix[-1]}
    _BATCH[group] = plan
    return plan


def _op_struct_type():
    from ._lib import PackOp
    return PackOp


def prefetch_packs() -> None:
    """After the optimizer step: rebuild every weight pack of the plan on the side stream, one by one
    in the order the forward will ask for them (the encoder's first, so the forward's first wait is
    short), each behind its own event.  (Batched avc_pack_batch launches measured +0.12 ms per C2
    step here: their few per-group events let the next forward start later; the recorded step
    rewrites its frozen packs in place with them, repack_in_place.)"""
    side = _SINK["side"]
    if side is None or not _PLAN:
        return
    side_raw = side.cuda_stream
    stream_wait(side_raw, ev_record())
    with _OnStream(side), torch.no_grad():
        for ref in list(_PLAN):
            c = ref()
            if c is None:
                _PLAN.remove(ref)
                continue
            if not c.used:  # only built inside a captured forward graph, which rebuilds it itself
                continue
            c.used = False
            key = _pack_key(c.params)
            if key == c.key:
                continue
            val = c.build()
            c.pending = (key, val, ev_token(side_raw))


def _need(t):
    return t is not None and t.requires_grad


# =============================================================================== plain conv helpers
def conv_pack_ops(w, val):
    """Batched-pack ops (avc_pack_batch) rewriting (Wf, Wd) of conv weight w in place."""
    from ._lib import PACK_CONV_D, PACK_CONV_F

    Co, Ci, Kw = w.shape
    return [{"src": w.data_ptr(), "dst": t.data_ptr(), "kind": kind, "dtype": K._dt(t), "dims": (Co, Ci, Kw)}
            for t, kind in zip(val, (PACK_CONV_F, PACK_CONV_D))]


def conv_packs(cache, w):
    """(Wf [Co][Kw*Ci], Wd [Ci][Kw*Co]) in the compute dtype, rebuilt when w changes."""
    def build():
        dt = K.compute()
        return K.conv_pack(w, 0, dt), K.conv_pack(w, 1, dt)
    return cache.get([w], build, ops=lambda val: conv_pack_ops(w, val))


def conv_fwd(x, B, T_in, w, bias, pad, Wf, out=None):
    """Conv1d(stride 1) on frame-major x (B*T_in, Ci) -> (B*T_out, Co), T_out."""
    Co, Ci, Kw = w.shape
    T_out = T_in + 2 * pad - Kw + 1
    y = torch.empty(B * T_out, Co, device=x.device) if out is None else out
    K.gemm(B * T_out, Co, Kw * Ci, operand(x, Ci, window=(Kw, pad, T_out, T_in, Ci)), operand(Wf, Kw * Ci), y,
           bias=bias)
    return y, T_out


def conv_wgrad(dy, x, B, T_in, T_out, w, pad, into=None):
    """dW of a Conv1d, written by the GEMM epilogue straight into the [Co][Ci][K] layout
    (accumulated into `into`, e.g. the parameter's .grad, when given)."""
    Co, Ci, Kw = w.shape
    M = B * T_out
    halo = Kw == 5 and 2 * pad == Kw - 1 and T_in == T_out and Ci % 32 == 0 and M % T_out == 0
    sk = K.auto_split_k(Co, Kw * Ci, M)
    # the direct [Co][Ci][K] epilogue scatters its columns 4*Kw bytes apart: with split-K atomics
    # that is ~Kw x the atomic requests of the packed layout (measured +0.9 ms per C2 step), so
    # split products reduced by atomics go through the packed dWf and one unpack pass instead;
    # on the halo weight-gradient kernel (gemm_tt.hip: 5-tap 'same', Ci % 32 == 0) a product whose
    # partials the last split reduces (K.tt_splitk_reduced) stores the layout directly, 16-B runs
    if sk > 1 and Kw > 1 and not (halo and K.tt_splitk_reduced(sk)):
        dWf = torch.empty(Co, Kw * Ci, device=x.device)
        K.gemm(Co, Kw * Ci, M, operand(dy, Co, kstrided=True),
               operand(x, Ci, kstrided=True, window=(Kw, pad, T_out, T_in, Ci)), dWf, split_k=sk)
        return K.conv_grad_unpack(dWf, Co, Ci, Kw, into=into)
    dW = torch.empty(Co, Ci, Kw, device=x.device) if into is None else into
    K.gemm(Co, Kw * Ci, M, operand(dy, Co, kstrided=True),
           operand(x, Ci, kstrided=True, window=(Kw, pad, T_out, T_in, Ci)), dW.view(Co, Ci * Kw),
           split_k=sk, accumulate=into is not None, cperm=Kw)
    return dW


def conv_dgrad(dy, B, T_in, T_out, w, pad, Wd, n_dx=None):
    Co, Ci, Kw = w.shape
    n_dx = Ci if n_dx is None else n_dx
    dx = torch.empty(B * T_in, n_dx, device=dy.device)
    K.gemm(B * T_in, n_dx, Kw * Co, operand(dy, Co, window=(Kw, Kw - 1 - pad, T_in, T_out, Co)), operand(Wd, Kw * Co), dx)
    return dx


# =============================================================================== conv + BN
class ConvBNCore:
    """ConvNorm (Norm.py:4-37) + BatchNorm1d + activation, frame-major.

    act: K.ACT_* applied after BN (AutoVC order: conv -> BN -> act, AutoVC.py:50-51)."""

    def __init__(self, conv: torch.nn.Conv1d, bn: torch.nn.BatchNorm1d, act: int):
        self.conv, self.bn, self.act = conv, bn, act
        self.pad = conv.padding[0]
        self.cache = PackCache()
        # running-statistics updates per forward: 2 when one forward stands for two identical
        # reference passes (the *_Adjust models' c_org / c_trg Adjust calls)
        self.stat_updates = 1

    def packs(self):
        w = self.conv.weight

        def build():
            dt = K.compute()
            return K.conv_pack(w, 0, dt), K.conv_pack(w, 1, dt)
        return self.cache.get([w], build, ops=lambda val: conv_pack_ops(w, val))

    def forward(self, x, B, T_in, residual=None, out_bf16=False):
        """out_bf16 (bf16 compute only): the activation is returned as a bf16 tensor -- for a
        layer whose output is read by bf16 GEMMs alone (the next conv / an LSTM input
        projection); its gradient then arrives in bf16 too.  In bf16 mode the conv output y
        (kept for the BN backward) is stored in bf16; the BN statistics come from the fp32
        accumulators in the GEMM epilogue."""
        Co, Ci, Kw = self.conv.weight.shape
        T_out = T_in + 2 * self.pad - Kw + 1
        Wf, _ = self.packs()
        x = K.twin(x)
        xop, wop = operand(x, Ci, window=(Kw, self.pad, T_out, T_in, Ci)), operand(Wf, Kw * Ci)
        return self.conv_bn_act(xop, wop, Kw * Ci, B * T_out, T_out, x.device, residual, out_bf16)

    def conv_bn_act(self, xop, wop, Kdim, M, T_out, dev, residual=None, out_bf16=False, row_bias=None):
        """The conv GEMM (operands given) + BatchNorm (statistics from the epilogue) + activation."""
        conv, bn = self.conv, self.bn
        Co = conv.weight.shape[0]
        bf = K.compute() == K.BF16
        y = torch.empty(M, Co, device=dev, dtype=torch.bfloat16 if bf else torch.float32)
        a = None
        if bn.training:
            # batch statistics from the epilogue, finalized by the GEMM's last row tiles; the
            # running statistics take stat_updates updates (the *_Adjust double pass)
            partial = K.bn_partial_buffer(M, Co, dev)
            nbt = bn.num_batches_tracked if bn.track_running_stats else None
            mom = bn.momentum if bn.momentum is not None else 0.1
            stats = K.gemm(M, Co, Kdim, xop, wop, y, bias=conv.bias, bn_partial=partial,
                           bn_fin=(bn.weight, bn.bias, bn.running_mean, bn.running_var, nbt, mom, bn.eps,
                                   self.stat_updates), row_bias=row_bias)
        else:
            K.gemm(M, Co, Kdim, xop, wop, y, bias=conv.bias, row_bias=row_bias)
            stats = K.bn_eval(bn.running_mean, bn.running_var, bn.weight, bn.bias, bn.eps)
        mean, rstd, scale, shift = stats
        if a is None:
            a = K.bn_apply(y, scale, shift, self.act, residual, out_bf16=out_bf16 and bf and residual is None)
        return a, (y, mean, rstd, T_out)

    def bn_grad(self, dA, saved, self_link=None):
        """BatchNorm + activation backward: dy (bf16 in bf16 mode) and, outside sink mode, the
        (dgamma, dbeta, conv-bias) gradients (sink mode: accumulated into .grad)."""
        y, mean, rstd, _ = saved
        if not self.bn.training:
            raise NotImplementedError("backward through eval-mode BatchNorm is not supported")
        conv, bn = self.conv, self.bn
        dy_bf16 = K.compute() == K.BF16
        if self_link is not None and self_link.coef is not None:
            # statistics (and the parameter gradients) came from the consumer's GEMM epilogue, and
            # dy too (avc_bnb_args.dy_bf16) when the link asked for it
            if dA.data_ptr() != self_link.dA_ptr:
                raise RuntimeError("fused BatchNorm backward: dL/da is not the linked consumer's data gradient "
                                   "(the output was used twice?)")
            dy = self_link.dy if self_link.dy is not None else K.bn_bwd_apply(dA, y, self_link.coef, self.act,
                                                                              dy_bf16=dy_bf16)
            dgamma, dbeta, dbias = self_link.grads
            self_link.coef = self_link.dy = None
            return dy, dgamma, dbeta, dbias
        into = (_grad_of(bn.weight), _grad_of(bn.bias), _grad_of(conv.bias)) if _SINK["on"] else None
        # act' from the recomputed pre-activation: the activation output `a` is not re-read
        # bf16 mode: dy feeds the two bf16 GEMMs below only -> stored in bf16 alone
        dy, dgamma, dbeta, dbias = K.bn_bwd(dA, None, y, mean, rstd, bn.weight, self.act, into=into,
                                            beta=bn.bias, dy_bf16=dy_bf16)
        return dy, dgamma, dbeta, dbias

    def fold_packs(self, nm, cp):
        """Packs of the conv0 fold (fold.hip): the first nm input channels as Wf [Co][K*cp] and
        Wd [nm][K*Co], the rest (the broadcast speaker embedding) as We [K*Co][Ci - nm]."""
        w = self.conv.weight
        if not hasattr(self, "fold_cache"):
            self.fold_cache = PackCache()

        Co, Ci, Kw = w.shape
        slices = ((0, nm, cp, 0), (0, nm, nm, 1), (nm, Ci - nm, Ci - nm, 2))

        def build():
            dt = K.compute()
            # (an fp32 speaker term on the generic fp32 kernel cost 51 us for this 64-row product)
            return tuple(K.conv_pack_slice(w, ci0, cn, cpad, mode, dt) for ci0, cn, cpad, mode in slices)

        def ops(val):  # the same three slices inside the batched repack (avc_pack_batch CONV_SLICE)
            from ._lib import PACK_CONV_SLICE

            return [{"src": w.data_ptr(), "dst": t.data_ptr(), "kind": PACK_CONV_SLICE, "dtype": K._dt(t),
                     "dims": (Co, Ci, Kw), "slice": sl} for t, sl in zip(val, slices)]
        return self.fold_cache.get([w], build, ops=ops)

    def backward(self, dA, x, a, saved, B, T_in, n_dx, self_link=None, prev_link=None):
        """self_link: this layer's BnbLink (its BN backward statistics may already have been
        computed by the consumer's data-gradient GEMM); prev_link: the link of the conv + BN
        layer that produced x, whose statistics this layer's data-gradient GEMM computes."""
        T_out = saved[3]
        conv = self.conv
        Co, Ci, Kw = conv.weight.shape
        M = B * T_out
        sink = _SINK["on"]
        dy, dgamma, dbeta, dbias = self.bn_grad(dA, saved, self_link)

        def wgrad():
            return conv_wgrad(dy, x, B, T_in, T_out, conv.weight, self.pad,
                              into=_grad_of(conv.weight) if sink else None)
        ev = mark()
        dx = None
        if n_dx:
            _, Wd = self.packs()
            dx = torch.empty(B * T_in, n_dx, device=x.device, dtype=x.dtype)
            bnb = prev_link.gemm_args(B * T_in, n_dx, sink) if prev_link is not None and n_dx == Ci else None
            K.gemm(B * T_in, n_dx, Kw * Co, operand(dy, Co, window=(Kw, Kw - 1 - self.pad, T_in, T_out, Co)),
                   operand(Wd, Kw * Co), dx, bnb=bnb,
                   **({"bnb_dy": prev_link.dy} if bnb is not None and prev_link.dy is not None else {}))
            if bnb is not None:
                prev_link.dA_ptr = dx.data_ptr()
        if sink and main_wgrad(conv.weight, last=not n_dx):
            # the tail of the backward: on the main stream, right behind the data gradient
            if not _ABLATE_WGRAD:
                wgrad()
            dW = dgamma = dbeta = dbias = None
        elif sink:
            with _Side(ev) as sd:
                sd.keep(dy, x)
                if not _ABLATE_WGRAD:
                    wgrad()
                side_wrote(conv.weight)
            dW = dgamma = dbeta = dbias = None
        else:
            dW = wgrad()
        return dx, dW, dbias, dgamma, dbeta


class BnbLink:
    """A conv + BN + act layer whose output feeds ONE consumer conv_bn (fuse_prev=True at the call
    site, where the model code guarantees the single use): the consumer's data-gradient GEMM
    computes this layer's BatchNorm backward statistics and parameter gradients in its epilogue
    (avc_gemm_bnb), and this layer's backward runs only the apply pass -- the separate reduce
    and finalize launches of nn.BatchNorm1d.backward's statistics (AutoVC.py:38,91,138,154,169)
    are gone.  One-shot per forward."""

    __slots__ = ("core", "saved", "coef", "dA_ptr", "grads", "dy")

    def __init__(self, core, saved):
        self.core, self.saved = core, saved
        self.coef, self.dA_ptr, self.grads, self.dy = None, None, (None, None, None), None

    def gemm_args(self, M, C, sink):
        core = self.core
        y, mean, rstd, _ = self.saved
        if y.shape != (M, C):
            return None
        bn, conv = core.bn, core.conv
        dev = y.device
        if sink:
            dg, db, dbi = _grad_of(bn.weight), _grad_of(bn.bias), (_grad_of(conv.bias) if conv.bias is not None else None)
            self.grads = (None, None, None)
        else:
            dg, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
            dbi = torch.empty(C, device=dev) if conv.bias is not None else None
            self.grads = (dg, db, dbi)
        self.coef = torch.empty(6 * C, device=dev)
        # the layer's dy (bf16) from the same GEMM (avc_bnb_args.dy_bf16; on the halo conv: its epilogue)
        self.dy = None
        return (y, mean, rstd, bn.weight, bn.bias, core.act, self.coef, dg, db, dbi, int(sink))


def _links(ctx, x, core, a, saved, fuse_prev):
    """Forward bookkeeping of the fused BN-backward statistics (BnbLink), bf16 training only."""
    on = _BNB_ON and K.compute() == K.BF16 and core.bn.training
    # only where the consumer's data-gradient conv runs on the halo conv ring (utterance-aligned
    # 128-frame tiles, >= 128 channels): on gemm_conv's epilogue the fusion measured slower (round 2)
    Co = core.conv.weight.shape[0]
    ring_ok = saved[3] % 128 == 0 and Co >= 128 and Co % 32 == 0
    ctx.self_link = BnbLink(core, saved) if (on and ring_ok) else None
    on = on and ring_ok
    if on:
        a._bnb_link = ctx.self_link
    prev = getattr(x, "_bnb_link", None) if (on and fuse_prev) else None
    ctx.prev_link = prev if (prev is not None and prev.core.bn.training) else None


# the BN-backward statistics of a conv + BN layer in its consumer's data-gradient conv (the halo conv
# ring's ring_bnb_epilogue, aligned T only -- see _links): on since round 5 (C2 5.74 -> 5.67 ms,
# profiles/r5_bnb_ab.txt); "0": the separate reduce / finalize passes
_BNB_ON = os.environ.get("AVC_BNB", "1") != "0"
# (round 5 also applied BN + act inside the halo conv's epilogue behind a column-tile barrier: slower in
# the C2 step, ~12 us per conv against a 6 us apply pass, profiles/r5_bn_apply_fused_ab.txt; removed in
# round 6.  avc_bn_fin.apply_bf16 / avc_bnb_args.dy_bf16 still ask one GEMM call for the apply outputs,
# written by a pass after the GEMM.)


class _ConvBNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, core, B, T_in, residual, out_bf16, fuse_prev, w, b, gamma, beta):
        a, saved = core.forward(x, B, T_in, residual, out_bf16)
        ctx.core, ctx.B, ctx.T_in, ctx.saved = core, B, T_in, saved
        ctx.has_res = residual is not None
        ctx.save_for_backward(x, a)
        ctx.x16 = getattr(x, "_bf16", None)
        _links(ctx, x, core, a, saved, fuse_prev)
        return a

    @staticmethod
    def backward(ctx, dA):
        x, a = ctx.saved_tensors
        K.attach_twin(x, ctx.x16)
        dA = dA.contiguous()
        n_dx = x.shape[1] if ctx.needs_input_grad[0] else 0
        dx, dW, db, dg, dbe = ctx.core.backward(dA, x, a, ctx.saved, ctx.B, ctx.T_in, n_dx, self_link=ctx.self_link,
                                                prev_link=ctx.prev_link)
        dres = dA if ctx.has_res and ctx.needs_input_grad[4] else None
        return dx, None, None, None, dres, None, None, dW, db, dg, dbe


def conv_bn(core: ConvBNCore, x, B, T_in, residual=None, out_bf16=False, fuse_prev=False):
    """out_bf16: the caller feeds the result only to another conv_bn / lstm (bf16 storage in
    bf16 compute mode, see ConvBNCore.forward).  fuse_prev: x is the output of a conv_bn /
    enc_conv0 used by this layer alone -- its BatchNorm backward statistics ride on this layer's
    data-gradient GEMM (BnbLink)."""
    c, bn = core.conv, core.bn
    return _ConvBNFn.apply(x, core, B, T_in, residual, out_bf16, fuse_prev, c.weight, c.bias, bn.weight, bn.bias)


class _EncConv0Fn(torch.autograd.Function):
    """cat(mel, c_org broadcast) -> conv0 + BN + ReLU (AutoVC.py:46-51); dL/dmel via a
    data-gradient GEMM restricted to the 80 mel channels."""

    @staticmethod
    def forward(ctx, mel2d, emb, core, B, T, out_bf16, w, b, gamma, beta):
        x = K.enc_concat(mel2d, emb, B, T)
        a, saved = core.forward(x, B, T, None, out_bf16)
        ctx.core, ctx.B, ctx.T, ctx.saved, ctx.n_mel = core, B, T, saved, mel2d.shape[1]
        ctx.save_for_backward(x, a)
        ctx.x16 = getattr(x, "_bf16", None)
        _links(ctx, x, core, a, saved, False)
        return a

    @staticmethod
    def backward(ctx, dA):
        x, a = ctx.saved_tensors
        K.attach_twin(x, ctx.x16)
        # a trained speaker embedding (the *_Adjust variants feed Adjust's output here,
        # AutoVC_Adjust.py:179-181) takes the full-width data gradient, summed over time
        nm = ctx.n_mel
        demb_needed = ctx.needs_input_grad[1]
        n_dx = x.shape[1] if demb_needed else (nm if ctx.needs_input_grad[0] else 0)
        dx, dW, db, dg, dbe = ctx.core.backward(dA.contiguous(), x, a, ctx.saved, ctx.B, ctx.T, n_dx,
                                                self_link=ctx.self_link)
        demb = None
        if demb_needed:
            demb = K.segsum(dx[:, nm:], ctx.B, ctx.T, x.shape[1] - nm, ld=x.shape[1])
            dx = dx[:, :nm] if ctx.needs_input_grad[0] else None
        return dx, demb, None, None, None, None, dW, db, dg, dbe


class _EncConv0FoldFn(torch.autograd.Function):
    """The same layer with the speaker half folded out of the frames (fold.hip,
    AutoVC.py:46-51): conv0 runs on the mel channels (zero-padded to a multiple of 32) and the
    broadcast embedding's contribution E = c_org . We (B x K*Co) enters as a per-(utterance,
    edge class) row bias of the GEMM epilogue, before the BatchNorm statistics.  Backward: dy's
    per-utterance column sums over each tap's valid frames (Sdy) give the embedding half of
    dW (a K = B product per tap) and, for a trained embedding, dc_org = Sdy . We; the mel half
    of dW and dL/dmel are the usual halo-conv products over the padded mel channels."""

    @staticmethod
    def forward(ctx, mel2d, emb, core, B, T, out_bf16, w, b, gamma, beta):
        Co, Ci, Kw = core.conv.weight.shape
        nm, pad = mel2d.shape[1], core.pad
        de, cp = Ci - nm, -(-nm // 32) * 32
        Wmf, _, We = core.fold_packs(nm, cp)
        dev = mel2d.device
        xm = K.pad_cols(mel2d, cp, dtype=K.compute())
        # the speaker term's edge table depends on emb and the weights only: the encoder re-pass on
        # mel_postnet (same c_org, same weights) reuses the first pass's table (a recorded step replays
        # the reuse; a refilled emb bumps its version, an Adam step the pack epoch)
        key = (_pack_key([core.conv.weight]), emb._version, B, T)
        hit = getattr(core, "_edge", None)
        if hit is not None and hit[0]() is emb and hit[1] == key:
            S = hit[2]
        else:
            # a fresh compute-dtype copy of emb, never attached to it: a caller may refill emb in
            # place (a captured step fed through the same input tensors), a cached twin would go stale
            e = K.convert(emb, K.BF16) if K.compute() == K.BF16 else emb
            E = torch.empty(B, Kw * Co, device=dev)
            K.gemm(B, Kw * Co, de, operand(e, de), operand(We, de), E)
            S = K.conv_edge_table(E, B, Co, Kw, T, pad)
            core._edge = (weakref.ref(emb), key, S)
        a, saved = core.conv_bn_act(operand(xm, cp, window=(Kw, pad, T, T, cp)), operand(Wmf, Kw * cp), Kw * cp,
                                    B * T, T, dev, None, out_bf16, row_bias=(S, T, pad))
        ctx.core, ctx.B, ctx.T, ctx.saved, ctx.dims = core, B, T, saved, (nm, de, cp)
        ctx.save_for_backward(xm, emb, a)
        _links(ctx, xm, core, a, saved, False)
        return a

    @staticmethod
    def backward(ctx, dA):
        xm, emb, a = ctx.saved_tensors
        core, B, T = ctx.core, ctx.B, ctx.T
        nm, de, cp = ctx.dims
        conv = core.conv
        Co, Ci, Kw = conv.weight.shape
        pad, M = core.pad, B * T
        sink = _SINK["on"]
        dy, dgamma, dbeta, dbias = core.bn_grad(dA.contiguous(), ctx.saved, ctx.self_link)
        _, Wmd, We = core.fold_packs(nm, cp)
        Sdy = K.conv_edge_colsum(dy, B, T, Co, Kw, pad)  # (B*Kw, Co): dy summed over each tap's valid frames
        ev = mark()
        dmel = demb = None
        if ctx.needs_input_grad[0]:  # the encoder re-pass: dL/d(mel_postnet)
            dmel = torch.empty(M, nm, device=dy.device)
            K.gemm(M, nm, Kw * Co, operand(dy, Co, window=(Kw, Kw - 1 - pad, T, T, Co)), operand(Wmd, Kw * Co), dmel)
        if ctx.needs_input_grad[1]:  # a trained embedding (the *_Adjust variants)
            demb = torch.empty(B, de, device=dy.device)
            K.gemm(B, de, Kw * Co, operand(Sdy, Kw * Co), operand(We, de, kstrided=True), demb)

        def wgrad(gw, acc):
            """dW into gw: accumulated (acc) or written -- the mel half [0, nm) and the embedding
            half [nm, nm + de) of the input channels cover all of them."""
            dWm = torch.empty(Co, Kw * cp, device=dy.device)
            K.gemm(Co, Kw * cp, M, operand(dy, Co, kstrided=True),
                   operand(xm, cp, kstrided=True, window=(Kw, pad, T, T, cp)), dWm,
                   split_k=K.auto_split_k(Co, Kw * cp, M))
            K.conv_grad_unpack_slice(dWm, Kw * cp, cp, gw, 0, nm, accumulate=acc)
            # embedding half, one K = B product per tap: dWe[co][k][ci] = sum_b Sdy[b][k][co] emb[b][ci]
            dWe = torch.empty(Co, Kw * de, device=dy.device)
            K.gemm(Co, de, B, operand(Sdy, Kw * Co, kstrided=True, batch_stride=Co),
                   operand(emb, de, kstrided=True), dWe, ldc=Kw * de, batch=Kw, c_batch_stride=de)
            K.conv_grad_unpack_slice(dWe, Kw * de, de, gw, nm, de, accumulate=acc)
            return gw
        if sink and main_wgrad(conv.weight, last=dmel is None and demb is None):
            # the tail of the backward: on the main stream (see ConvBNCore.backward)
            if not _ABLATE_WGRAD:
                wgrad(_grad_of(conv.weight), True)
            dW = dgamma = dbeta = dbias = None
        elif sink:
            with _Side(ev) as sd:
                sd.keep(dy, xm, Sdy, emb)
                if not _ABLATE_WGRAD:
                    wgrad(_grad_of(conv.weight), True)
                side_wrote(conv.weight)
            dW = dgamma = dbeta = dbias = None
        else:
            dW = wgrad(torch.empty_like(conv.weight), False)
        return dmel, demb, None, None, None, None, dW, dbias, dgamma, dbeta


# the speaker-half fold of the encoder's first conv (AVC_FOLD=0: the concat forms of conv0 and of the
# decoder's lstm1 input, A/B and parity diagnostics)
_FOLD = os.environ.get("AVC_FOLD", "1") != "0"


def enc_conv0(core, mel2d, emb, B, T, out_bf16=False):
    c, bn = core.conv, core.bn
    Kw = c.weight.shape[2]
    if _FOLD and Kw == 2 * core.pad + 1 and T > 2 * core.pad and c.weight.shape[1] > mel2d.shape[1]:
        return _EncConv0FoldFn.apply(mel2d, emb, core, B, T, out_bf16, c.weight, c.bias, bn.weight, bn.bias)
    return _EncConv0Fn.apply(mel2d, emb, core, B, T, out_bf16, c.weight, c.bias, bn.weight, bn.bias)


# =============================================================================== LSTM
class LSTMLayerCore:
    """One layer (both directions) of nn.LSTM(batch_first=True), h0 = c0 = 0."""

    def __init__(self, mod, layer: int):
        self.mod, self.layer = mod, layer
        self.dirs = 2 if mod.bidirectional else 1
        self.H = mod.hidden_size
        self.cache = PackCache()

    def params(self):
        out = []
        for sfx in (["", "_reverse"] if self.dirs == 2 else [""]):
            for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh"):
                out.append(getattr(self.mod, f"{n}_l{self.layer}{sfx}"))
        return out

    def packs(self):
        ps = self.params()

        def build():
            dt = K.compute()
            H, dirs = self.H, self.dirs
            In = ps[0].shape[1]
            dev = ps[0].device
            tdt = K.compute_torch_dtype()
            wih = torch.empty(dirs * 4 * H, In, device=dev, dtype=tdt)
            bsum = torch.empty(dirs * 4 * H, device=dev)
            large = H > 64
            whh = torch.empty(dirs * 4 * H, H, device=dev, dtype=tdt if large else torch.float32)
            whh_t = torch.empty(dirs * H, 4 * H, device=dev, dtype=tdt) if large else None
            # W_ih^T (In x dirs*4H) makes the input-gradient GEMM K-contiguous in both operands
            wih_t = torch.empty(In, dirs * 4 * H, device=dev, dtype=tdt)
            for d in range(dirs):
                w_ih, w_hh, b_ih, b_hh = ps[4 * d: 4 * d + 4]
                K.convert(w_ih, dt, out=wih[d * 4 * H:(d + 1) * 4 * H])
                K.add(b_ih, b_hh, out=bsum[d * 4 * H:(d + 1) * 4 * H])
                K.convert(w_hh, dt if large else K.F32, out=whh[d * 4 * H:(d + 1) * 4 * H])
                if large:
                    K.transpose(w_hh, dt, out=whh_t[d * H:(d + 1) * H])
            for d in range(dirs):
                K.transpose(ps[4 * d], dt, out=wih_t[:, d * 4 * H:], ld_out=dirs * 4 * H)
            return wih, bsum, whh, whh_t, wih_t

        def ops(val):
            from ._lib import PACK_ADD, PACK_COPY, PACK_TRANSPOSE

            wih, bsum, whh, whh_t, wih_t = val
            H, dirs = self.H, self.dirs
            G = 4 * H
            out = []
            for d in range(dirs):
                w_ih, w_hh, b_ih, b_hh = ps[4 * d: 4 * d + 4]
                In = w_ih.shape[1]
                out.append({"src": w_ih.data_ptr(), "dst": wih[d * G:].data_ptr(), "kind": PACK_COPY,
                            "dtype": K._dt(wih), "dims": (G * In,)})
                out.append({"src": b_ih.data_ptr(), "src2": b_hh.data_ptr(), "dst": bsum[d * G:].data_ptr(),
                            "kind": PACK_ADD, "dtype": K.F32, "dims": (G,)})
                out.append({"src": w_hh.data_ptr(), "dst": whh[d * G:].data_ptr(), "kind": PACK_COPY,
                            "dtype": K._dt(whh), "dims": (G * H,)})
                if whh_t is not None:
                    out.append({"src": w_hh.data_ptr(), "dst": whh_t[d * H:].data_ptr(), "kind": PACK_TRANSPOSE,
                                "dtype": K._dt(whh_t), "dims": (G, H), "ld": G})
                out.append({"src": w_ih.data_ptr(), "dst": wih_t[:, d * G:].data_ptr(), "kind": PACK_TRANSPOSE,
                            "dtype": K._dt(wih_t), "dims": (G, In), "ld": dirs * G})
            return out
        return self.cache.get(ps, build, ops=ops)

    def forward(self, x, B, T):
        H, dirs = self.H, self.dirs
        In = x.shape[1]
        wih, bsum, whh, _, _ = self.packs()
        x = K.twin(x)
        xproj = torch.empty(B * T, dirs * 4 * H, device=x.device)
        K.gemm(B * T, dirs * 4 * H, In, operand(x, In), operand(wih, In), xproj, bias=bsum)
        hbuf = None
        if H > 64 and K.compute() == K.BF16:
            hbuf = K.lstm_scratch(B, H, dirs, x.device)
        h, c, g = K.lstm_fwd(xproj, whh, B, T, H, dirs, hbuf)
        return h, (c, g)

    def backward(self, dh, x, h, saved, B, T, need_dx, dg=None, dbp=None):
        """dg: the gate gradients when a fused launch already produced them (the lstm2 wavefront:
        bf16 only when it also gave dbp, the (groups, 4H) partial sums of dg whose column sums are
        the bias gradients)."""
        c, g = saved
        H, dirs = self.H, self.dirs
        In = x.shape[1]
        wih, _, whh, whh_t, wih_t = self.packs()
        if dg is None:
            dg = K.lstm_bwd(dh, h, c, g, whh if H <= 64 else None, whh_t, B, T, H, dirs)
        G = dirs * 4 * H
        M = B * T
        sink = _SINK["on"]
        ps = self.params()

        K.twin(dg)  # bf16 operand copy for the GEMMs (already there on the persistent path)
        # GEMM operand sources: the bf16 twins when present (column views of them keep bf16)
        dg_op = getattr(dg, "_bf16", None) if K.compute() == K.BF16 else None
        dg_op = dg if dg_op is None else dg_op
        h_op = getattr(h, "_bf16", None) if K.compute() == K.BF16 else None
        h_op = h if h_op is None else h_op

        def wgrads():
            grads = []
            for d in range(dirs):
                w_ih, w_hh, b_ih, b_hh = ps[4 * d: 4 * d + 4]
                dgd = dg_op if dirs == 1 else dg_op[:, d * 4 * H:]
                dwih = _grad_of(w_ih) if sink else torch.empty(4 * H, In, device=x.device)
                K.gemm(4 * H, In, M, operand(dgd, G, kstrided=True), operand(x, In, kstrided=True), dwih,
                       split_k=K.auto_split_k(4 * H, In, M), accumulate=sink)
                dwhh = _grad_of(w_hh) if sink else torch.empty(4 * H, H, device=x.device)
                shift = 1 if d == 0 else -1
                hd = h_op if dirs == 1 else h_op[:, d * H:]
                K.gemm(4 * H, H, M, operand(dgd, G, kstrided=True),
                       operand(hd, dirs * H, kstrided=True, window=(1, shift, T, T, H)), dwhh,
                       split_k=K.auto_split_k(4 * H, H, M), accumulate=sink)
                # bias gradients: column sums of dG, or of the wavefront's per-group partials
                dg32, rows = (dg if dirs == 1 else dg[:, d * 4 * H:], M) if dbp is None else (dbp, dbp.shape[0])
                if sink:
                    K.colsum(dg32, rows, 4 * H, ld=G, out=_grad_of(b_ih), out2=_grad_of(b_hh), accumulate=True)
                    continue
                dbd = K.colsum(dg32, rows, 4 * H, ld=G)
                # b_ih and b_hh receive the same gradient but must not share storage
                grads += [dwih, dwhh, dbd, K.convert(dbd, K.F32)]
            return grads
        ev = mark()
        dx = None
        if need_dx:
            dx = torch.empty(M, In, device=x.device, dtype=x.dtype)  # bf16 for a bf16-stored input
            K.gemm(M, In, G, operand(dg, G), operand(wih_t, G), dx)
        if sink:
            with _Side(ev) as sd:
                sd.keep(dg, x, h, dg_op, h_op, dbp)
                if not _ABLATE_WGRAD:
                    wgrads()
            grads = [None] * (4 * dirs)
        else:
            grads = wgrads()
        return dx, grads


class _LSTMLayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, core, B, T, *params):
        h, saved = core.forward(x, B, T)
        ctx.core, ctx.B, ctx.T, ctx.saved = core, B, T, saved
        ctx.save_for_backward(x, h)
        # saved tensors come back as new Python objects: carry the bf16 twins explicitly
        ctx.twins = (getattr(x, "_bf16", None), getattr(h, "_bf16", None))
        return h

    @staticmethod
    def backward(ctx, dh):
        x, h = ctx.saved_tensors
        K.attach_twin(x, ctx.twins[0])
        K.attach_twin(h, ctx.twins[1])
        dx, grads = ctx.core.backward(dh.contiguous(), x, h, ctx.saved, ctx.B, ctx.T, ctx.needs_input_grad[0])
        return (dx, None, None, None, *grads)


def _pair_ok(cores, x, B):
    """Two stacked unidirectional layers that the one-launch wavefront kernel takes."""
    if len(cores) != 2 or _PAIR_OFF or K.compute() != K.BF16:
        return False
    c0, c1 = cores
    return (c0.dirs == 1 and c1.dirs == 1 and c0.H == c1.H and x.is_cuda
            and K.lstm2_persistent(B, c0.H, c1.params()[0].shape[1]))


class _LSTMPairFn(torch.autograd.Function):
    """Two stacked layers of one nn.LSTM (decoder lstm2, AutoVC.py:96,110): forward as ONE
    wavefront launch (avc_lstm2_fwd; layer 1's input projection inside the recurrence), backward
    layer by layer exactly as two _LSTMLayerFn nodes would run it."""

    @staticmethod
    def forward(ctx, x, c0, c1, B, T, *params):
        H = c0.H
        In = x.shape[1]
        wih0, bsum0, whh0, _, _ = c0.packs()
        wih1, bsum1, whh1, _, _ = c1.packs()
        x = K.twin(x)
        xproj = torch.empty(B * T, 4 * H, device=x.device)
        K.gemm(B * T, 4 * H, In, operand(x, In), operand(wih0, In), xproj, bias=bsum0)
        h0, cs0, g0, h1, cs1, g1 = K.lstm2_fwd(xproj, whh0, wih1, whh1, bsum1, B, T, H)
        ctx.cores, ctx.B, ctx.T, ctx.saved = (c0, c1), B, T, ((cs0, g0), (cs1, g1))
        ctx.save_for_backward(x, h0, h1)
        ctx.twins = (getattr(x, "_bf16", None), h0._bf16, h1._bf16)
        return h1

    @staticmethod
    def backward(ctx, dh1):
        x, h0, h1 = ctx.saved_tensors
        for t, tw in zip((x, h0, h1), ctx.twins):
            K.attach_twin(t, tw)
        c0, c1 = ctx.cores
        B, T, H = ctx.B, ctx.T, c0.H
        if _PAIR_BWD and K.lstm2_bwd_persistent(B, H):
            # both layers in one wavefront launch (avc_lstm2_bwd): dG1 W_ih1 inside the recurrence
            (cs0, gs0), (cs1, gs1) = ctx.saved
            wt0 = c0.packs()[3]
            _, _, _, wt1, wti1 = c1.packs()
            # bf16 dG only (the GEMM operands), the bias gradients from the kernel's per-group partials
            # (ABI 28; the fp32-dG form of the same kernel is held against it in test_gpu_lstm2_bwd.py)
            dg0, dg1, dbp = K.lstm2_bwd(dh1.contiguous(), cs0, gs0, cs1, gs1, wt0, wti1, wt1, B, T, H,
                                        fp32=False, db=True)
            dbp0, dbp1 = dbp[0], dbp[1]
            _, g1 = c1.backward(None, h0, h1, ctx.saved[1], B, T, False, dg=dg1, dbp=dbp1)
            dx, g0 = c0.backward(None, x, h0, ctx.saved[0], B, T, ctx.needs_input_grad[0], dg=dg0, dbp=dbp0)
            return (dx, None, None, None, None, *g0, *g1)
        dh0, g1 = c1.backward(dh1.contiguous(), h0, h1, ctx.saved[1], B, T, True)
        dx, g0 = c0.backward(dh0, x, h0, ctx.saved[0], B, T, ctx.needs_input_grad[0])
        return (dx, None, None, None, None, *g0, *g1)


_PAIR_OFF = bool(os.environ.get("AVC_LSTM2_OFF"))
# the pair's backward as one wavefront launch (avc_lstm2_bwd; C2 5.83 -> 5.81 ms, isolated 1127 -> ~1050 us,
# profiles/r5_lstm2_bwd_wavefront.txt); "0": two single-layer launches + the dX1 GEMM
_PAIR_BWD = os.environ.get("AVC_LSTM2_BWD", "1") != "0"


def lstm(mod, cores, x, B, T):
    if _pair_ok(cores, x, B):
        return _LSTMPairFn.apply(x, cores[0], cores[1], B, T, *cores[0].params(), *cores[1].params())
    for core in cores:
        x = _LSTMLayerFn.apply(x, core, B, T, *core.params())
    return x


class _LSTM1FoldFn(torch.autograd.Function):
    """Decoder lstm1 on cat(code expansion, c_trg broadcast) (AutoVC.py:96,103,197-204) with the
    input projection folded per code and per utterance: W_ih . [code_j ; e] + b =
    Wc . code_j + (We . e + b), computed once per code instead of a (B*T, cd+de) concat and its
    B*T x 4H x (cd+de) GEMM.  On the persistent path (bf16) that is ONE GEMM over the (B*nc, cd+de)
    rows [code_j ; e_b] (avc_code_cat) and the recurrence reads row b*nc + t/(T/nc) itself
    (avc_lstm_fwd_fold); elsewhere a per-code and a per-utterance GEMM expanded to the B*T frames
    (avc_expand_codes).  The backward is folded the same way: the gate gradients dG are summed over
    each code's frames (S_code; inside the persistent recurrence, avc_lstm_bwd_fold) and each
    utterance (S_utt) first, then
      dcodes = S_code . Wc,  dc_trg = S_utt . We,  dWc = S_code^T codes,  dWe = S_utt^T c_trg
      (= dW_ih = S_code^T [codes ; c_trg] over the code rows on the persistent path),
      db_ih = db_hh = colsum(S_code).
    `hook` (nullable) runs once every decoder / postnet gradient has been enqueued (the
    training step's overlapped decoder-slice all-reduce and Adam, train.py)."""

    @staticmethod
    def forward(ctx, codes, emb, core, B, T, nc, cd, hook, *params):
        H = core.H
        G = 4 * H
        de = emb.shape[1]
        In = cd + de
        wih, bsum, whh, _, _ = core.packs()
        dev = codes.device
        hbuf = K.lstm_scratch(B, H, 1, dev) if H > 64 and K.compute() == K.BF16 else None
        xcat = None
        if hbuf is not None and T % nc == 0 and K.lstm_persistent_fwd(B, H, 1) and K.lstm_persistent_bwd(B, H, 1):
            # one row per code, [code_j ; c_trg_b] in bf16: ONE GEMM gives every code's projection
            # incl. the per-utterance half and the bias, and the recurrence reads row b*nc + t/(T/nc)
            # itself (no (B*T, 4H) expansion)
            xcat = K.code_cat(codes, emb, B, nc, cd)
            pcode = torch.empty(B * nc, G, device=dev)
            K.gemm(B * nc, G, In, operand(xcat, In), operand(wih, In), pcode, bias=bsum)
            h, c, g = K.lstm_fwd_fold(pcode, nc, whh, B, T, H, hbuf)
        else:
            c2 = codes.reshape(B * nc, cd)
            pc = torch.empty(B * nc, G, device=dev)
            K.gemm(B * nc, G, cd, operand(c2, cd), operand(wih, In), pc)
            pe = torch.empty(B, G, device=dev)
            K.gemm(B, G, de, operand(emb, de), operand(wih[:, cd:], In), pe, bias=bsum)
            xproj = K.expand_codes(pc, pe, B, T, nc)
            h, c, g = K.lstm_fwd(xproj, whh, B, T, H, 1, hbuf)
        ctx.core, ctx.args, ctx.hook = core, (B, T, nc, cd), hook
        ctx.saved = (c, g, xcat)
        ctx.save_for_backward(codes, emb, h)
        ctx.h16 = getattr(h, "_bf16", None)
        return h

    @staticmethod
    def backward(ctx, dh):
        codes, emb, h = ctx.saved_tensors
        K.attach_twin(h, ctx.h16)
        core = ctx.core
        B, T, nc, cd = ctx.args
        c, g, xcat = ctx.saved
        H = core.H
        G = 4 * H
        de = emb.shape[1]
        In = cd + de
        _, _, whh, whh_t, wih_t = core.packs()
        dev = h.device
        M = B * T
        c2 = codes.reshape(B * nc, cd)
        if xcat is not None:
            # dG (bf16 only) and s_code = dG summed over each code's frames, both out of the recurrence
            dg, s_code = K.lstm_bwd_fold(dh.contiguous(), c, g, whh_t, B, T, H, nc)
        else:
            dg = K.lstm_bwd(dh.contiguous(), h, c, g, whh if H <= 64 else None, whh_t, B, T, H, 1)
            s_code = K.segsum(dg, B * nc, T // nc, G, ld=G)  # (B*nc, G): dG summed over each code's frames
        s_utt = None
        if xcat is None or ctx.needs_input_grad[1]:
            s_utt = K.segsum(s_code, B, nc, G, ld=G)  # (B, G): ... and over each utterance
        dcodes = demb = None
        # few output tiles, K = 4H: split K (atomic fp32 accumulation into zeroed outputs).  More
        # than two atomic partials make the sum order-dependent, so the fp32 parity mode keeps
        # these data gradients unsplit: its encoder gradients stay bit-reproducible (DP test)
        det = K.compute() == K.F32
        if ctx.needs_input_grad[0]:
            dcodes = torch.empty(B * nc, cd, device=dev)
            K.gemm(B * nc, cd, G, operand(s_code, G), operand(wih_t, G), dcodes,
                   split_k=1 if det else K.auto_split_k(B * nc, cd, G))
            dcodes = dcodes.view(B, nc * cd)
        if ctx.needs_input_grad[1]:
            demb = torch.empty(B, de, device=dev)
            K.gemm(B, de, G, operand(s_utt, G), operand(wih_t[cd:], G), demb,
                   split_k=1 if det else K.auto_split_k(B, de, G))
        sink = _SINK["on"]
        w_ih, w_hh, b_ih, b_hh = core.params()
        h_op = getattr(h, "_bf16", None) if K.compute() == K.BF16 else None
        h_op = h if h_op is None else h_op

        def wgrads():
            dwih = _grad_of(w_ih) if sink else torch.zeros(G, In, device=dev)
            if xcat is not None:  # sum_j s_code[b,j] c_trg[b] = s_utt[b] c_trg[b]: one product over the code rows
                K.gemm(G, In, B * nc, operand(s_code, G, kstrided=True), operand(xcat, In, kstrided=True), dwih,
                       ldc=In, accumulate=True, split_k=K.auto_split_k(G, In, B * nc))
            else:
                K.gemm(G, cd, B * nc, operand(s_code, G, kstrided=True), operand(c2, cd, kstrided=True), dwih,
                       ldc=In, accumulate=True, split_k=K.auto_split_k(G, cd, B * nc))
                K.gemm(G, de, B, operand(s_utt, G, kstrided=True), operand(emb, de, kstrided=True), dwih[:, cd:],
                       ldc=In, accumulate=True)
            dwhh = _grad_of(w_hh) if sink else torch.empty(G, H, device=dev)
            K.gemm(G, H, M, operand(dg, G, kstrided=True), operand(h_op, H, kstrided=True, window=(1, 1, T, T, H)),
                   dwhh, split_k=K.auto_split_k(G, H, M), accumulate=sink)
            if sink:
                K.colsum(s_code, B * nc, G, out=_grad_of(b_ih), out2=_grad_of(b_hh), accumulate=True)
                return [None] * 4
            dbd = K.colsum(s_code, B * nc, G)
            return [dwih, dwhh, dbd, K.convert(dbd, K.F32)]
        ev = mark()
        if sink:
            with _Side(ev) as sd:
                sd.keep(dg, h, h_op, s_code, s_utt, c2, emb, xcat)
                if not _ABLATE_WGRAD:
                    wgrads()
            grads = [None] * 4
        else:
            grads = wgrads()
        if ctx.hook is not None:
            ctx.hook()
        return (dcodes, demb, None, None, None, None, None, None, *grads)


def lstm1_folded(mod, core, codes, emb, B, T, nc, cd, hook=None):
    """Decoder lstm1 over cat(code expansion, emb) with the per-code / per-utterance input
    projection (see _LSTM1FoldFn); h (B*T, H)."""
    return _LSTM1FoldFn.apply(codes, emb, core, B, T, nc, cd, hook, *core.params())


# =============================================================================== linear
def copy_pack_ops(w, val):
    """Batched-pack op: val = w cast to the compute dtype."""
    from ._lib import PACK_COPY

    return [{"src": w.data_ptr(), "dst": val.data_ptr(), "kind": PACK_COPY, "dtype": K._dt(val), "dims": (w.numel(),)}]


def _linear_packs(cache, w):
    """(w, w^T) in the compute dtype: the forward's and the data gradient's K-contiguous B operands."""
    from ._lib import PACK_TRANSPOSE

    def build():
        return K.convert(w, K.compute()), K.transpose(w, K.compute())

    def ops(val):
        wc, wt = val
        return copy_pack_ops(w, wc) + [{"src": w.data_ptr(), "dst": wt.data_ptr(), "kind": PACK_TRANSPOSE,
                                        "dtype": K._dt(wt), "dims": tuple(w.shape), "ld": w.shape[0]}]
    return cache.get([w], build, ops=ops)


class _LinearFn(torch.autograd.Function):
    """LinearNorm (Norm.py:40-50) on frame-major rows."""

    @staticmethod
    def forward(ctx, x, w, b, cache):
        M, In = x.shape
        Out = w.shape[0]
        wc, _ = _linear_packs(cache, w)
        y = torch.empty(M, Out, device=x.device)
        # the bf16 twin from the GEMM's epilogue: the next layer's operand (the decoder projection feeds the
        # postnet's first conv) without a conversion pass
        y16 = torch.empty(M, Out, device=x.device, dtype=torch.bfloat16) if K.compute() == K.BF16 else None
        K.gemm(M, Out, In, operand(x, In), operand(wc, In), y, bias=b, c_bf16=y16)
        K.attach_twin(y, y16)
        ctx.cache = cache
        ctx.bias = b
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        M, In = x.shape
        Out = w.shape[0]
        sink = _SINK["on"]
        b = ctx.bias
        if K.compute() == K.BF16 and getattr(dy, "_bf16", None) is None:
            # a bf16 operand (the products round to bf16 either way) puts the data gradient on the
            # LDS-staged NT kernels instead of the register-staged fp32-operand path (29 -> ~13 us
            # for the decoder projection's 8192 x 1024 x 80), and the weight gradient on the TT kernel
            K.attach_twin(dy, K.convert(dy, K.BF16))

        def wgrad():
            dw = _grad_of(w) if sink else torch.empty(Out, In, device=x.device)
            K.gemm(Out, In, M, operand(dy, Out, kstrided=True), operand(x, In, kstrided=True), dw,
                   split_k=K.auto_split_k(Out, In, M), accumulate=sink)
            db = K.colsum(dy, M, Out, out=_grad_of(b) if sink else None, accumulate=sink)
            return dw, db
        ev = mark()
        dx = None
        if ctx.needs_input_grad[0]:
            _, wt = _linear_packs(ctx.cache, w)
            dx = torch.empty(M, In, device=x.device)
            K.gemm(M, In, Out, operand(dy, Out), operand(wt, Out), dx)
        if sink:
            with _Side(ev) as sd:
                sd.keep(dy, x)
                if not _ABLATE_WGRAD:
                    wgrad()
            dw = db = None
        else:
            dw, db = wgrad()
        return dx, dw, db, None


def linear(x, w, b, cache):
    return _LinearFn.apply(x, w, b, cache)


# =============================================================================== glue
class _CodesFn(torch.autograd.Function):
    """AutoVC.py:56-66 + torch.cat(codes, -1) (:195, :211)."""

    @staticmethod
    def forward(ctx, lo, B, T, D, freq):
        ctx.args = (B, T, D, freq)
        return K.codes_gather(lo, B, T, D, freq)

    @staticmethod
    def backward(ctx, dcodes):
        B, T, D, freq = ctx.args
        return K.codes_scatter(dcodes.contiguous(), B, T, D, freq), None, None, None, None


def codes(lo, B, T, D, freq):
    return _CodesFn.apply(lo, B, T, D, freq)


class _DecConcatFn(torch.autograd.Function):
    """Code expansion + c_trg broadcast concat (AutoVC.py:197-204)."""

    @staticmethod
    def forward(ctx, codes, emb, B, T, nc, cd):
        ctx.args = (B, T, nc, cd, emb.shape[1])
        return K.dec_concat(codes, emb, B, T, nc, cd)

    @staticmethod
    def backward(ctx, dout):
        B, T, nc, cd, de = ctx.args
        dout = dout.contiguous()
        dcodes = K.dec_concat_bwd(dout, B, T, nc, cd, de) if ctx.needs_input_grad[0] else None
        # c_trg trained through Adjust (AutoVC_Adjust.py:184-189): sum over the broadcast frames
        demb = K.segsum(dout[:, cd:], B, T, de, ld=cd + de) if ctx.needs_input_grad[1] else None
        return dcodes, demb, None, None, None, None


def dec_concat(codes, emb, B, T, nc, cd):
    return _DecConcatFn.apply(codes, emb, B, T, nc, cd)


# =============================================================================== layout
def _transpose_batched(x, B, R, C):
    """x viewed as B x [R][C] -> B x [C][R] (fp32), one launch (a per-utterance loop of transposes
    had cost the discriminator step 196 launches and 0.8 ms of GPU time)."""
    return K.transpose_batched(x, B, R, C)


class _BCTToFramesFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        B, C, T = x.shape
        ctx.shape = (B, C, T)
        return _transpose_batched(x.contiguous(), B, C, T).view(B * T, C)

    @staticmethod
    def backward(ctx, g):
        B, C, T = ctx.shape
        return _transpose_batched(g.contiguous(), B, T, C).view(B, C, T)


class _FramesToBCTFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, B, T):
        C = x.shape[1]
        ctx.shape = (B, C, T)
        return _transpose_batched(x.contiguous(), B, T, C).view(B, C, T)

    @staticmethod
    def backward(ctx, g):
        B, C, T = ctx.shape
        return _transpose_batched(g.contiguous(), B, C, T).view(B * T, C), None, None


def bct_to_frames(x):
    return _BCTToFramesFn.apply(x)


def frames_to_bct(x, B, T):
    return _FramesToBCTFn.apply(x, B, T)
