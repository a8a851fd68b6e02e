"""Per-step timeline of the persistent LSTM recurrences (avc_lstm_trace stamps) and event
timings of every recurrence kernel at the AutoVC shapes.

  python tools/lstm_trace.py [B] [T]

For each persistent launch (decoder lstm1 H=512, lstm2 H=1024; forward and backward) prints,
averaged over steps 1..T-1 and workgroups (us): wait = step start -> exchange complete,
prod = exchange complete -> product reduced, tail = product -> published, period = step to
step, and handoff = consumer's exchange complete - the LAST producer's publish in its group.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import autoformer_amd as A  # noqa: E402
from autoformer_amd import _lib  # noqa: E402
from autoformer_amd import kernels as K  # noqa: E402

A.set_compute("bf16")
dev = "cuda:0"
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
T = int(sys.argv[2]) if len(sys.argv) > 2 else 128


def ev_time(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def traced(fn, nwg):
    buf = torch.zeros(nwg * T * 4, dtype=torch.int64, device=dev)
    _lib.call("avc_lstm_trace", buf.data_ptr())
    try:
        fn()
        torch.cuda.synchronize()
    finally:
        _lib.call("avc_lstm_trace", None)
    return buf.cpu().numpy().reshape(nwg, T, 4).astype(np.float64) * 1e-2  # 100 MHz ticks -> us


def report(tag, st, ng):
    nwg = st.shape[0]
    s = slice(1, T)
    wait = (st[:, s, 1] - st[:, s, 0]).mean()
    prod = (st[:, s, 2] - st[:, s, 1]).mean()
    tail = (st[:, s, 3] - st[:, s, 2]).mean()
    period = np.diff(st[:, :, 0], axis=1)[:, 1:].mean()
    hand = []
    for g in range(ng):
        mem = [b for b in range(nwg) if b % ng == g]
        last_pub = st[mem, :-1, 3].max(axis=0)          # per step s: last member publish
        ready = st[mem, 1:, 1]                           # consumers' exchange complete at s+1
        hand.append((ready - last_pub[None, :]).mean())
    skew = (st[:, s, 3].max(axis=0) - st[:, s, 3].min(axis=0)).mean()
    span = st[:, -1, 3].max() - st[:, 0, 0].min()
    print(f"{tag}: span {span:8.1f} us = {span / T:5.2f} us/step | wait {wait:5.2f} prod {prod:5.2f} "
          f"tail {tail:5.2f} period {period:5.2f} handoff {np.mean(hand):5.2f} publish-skew {skew:5.2f}",
          flush=True)


for H in (1024, 512):
    G = 4 * H
    xproj = torch.randn(B * T, G, device=dev) * 0.1
    whh = (torch.randn(G, H, device=dev) * 0.02).bfloat16()
    whht = whh.t().contiguous()
    hbuf = K.lstm_scratch(B, H, 1, dev)
    ng = (B + 7) // 8
    nwg = ng * (H // 32)
    us = ev_time(lambda: K.lstm_fwd(xproj, whh, B, T, H, 1, hbuf))
    print(f"H={H} fwd events {us:8.1f} us ({us / T:5.2f} us/step)", flush=True)
    report(f"H={H} fwd", traced(lambda: K.lstm_fwd(xproj, whh, B, T, H, 1, hbuf), nwg), ng)
    h, c, g = K.lstm_fwd(xproj, whh, B, T, H, 1, hbuf)
    dh = torch.randn_like(h) * 0.1
    gbuf = K.lstm_bwd_scratch(B, H, 1, dev)
    usb = ev_time(lambda: K.lstm_bwd(dh, h, c, g, None, whht, B, T, H, 1, gbuf=gbuf))
    print(f"H={H} bwd events {usb:8.1f} us ({usb / T:5.2f} us/step)", flush=True)
    report(f"H={H} bwd", traced(lambda: K.lstm_bwd(dh, h, c, g, None, whht, B, T, H, 1, gbuf=gbuf), nwg), ng)
    assert K.lstm_timeout_flag(hbuf, B, H) == 0 and K.lstm_bwd_timeout_flag(gbuf, B, H) == 0

# decoder lstm2 as ONE two-layer wavefront launch (T + 1 ticks; stamps of ticks 0..T-1)
H = 1024
G = 4 * H
if K.lstm2_persistent(B, H, H):
    xproj = torch.randn(B * T, G, device=dev) * 0.1
    ws = [(torch.randn(G, H, device=dev) * 0.02).bfloat16() for _ in range(3)]
    bias1 = torch.randn(G, device=dev) * 0.1
    ng = (B + 15) // 16
    nwg = ng * (H // 16)
    us = ev_time(lambda: K.lstm2_fwd(xproj, *ws, bias1, B, T, H))
    print(f"lstm2 wavefront fwd events {us:8.1f} us ({us / (T + 1):5.2f} us/tick, 2 layers)", flush=True)
    report("lstm2 wavefront fwd", traced(lambda: K.lstm2_fwd(xproj, *ws, bias1, B, T, H), nwg), ng)

# encoder BiLSTM (small-H kernels, both directions in one launch)
H = 44
xproj = torch.randn(B * T, 2 * 4 * H, device=dev) * 0.1
whh = torch.randn(2 * 4 * H, H, device=dev) * 0.1
us = ev_time(lambda: K.lstm_fwd(xproj, whh, B, T, H, 2))
h, c, g = K.lstm_fwd(xproj, whh, B, T, H, 2)
dh = torch.randn_like(h) * 0.1
usb = ev_time(lambda: K.lstm_bwd(dh, h, c, g, whh, None, B, T, H, 2))
print(f"BiLSTM H=44 fwd {us:7.1f} us ({us / T:4.2f}/step)  bwd {usb:7.1f} us ({usb / T:4.2f}/step)", flush=True)

# BiLSTM per-step phases (TRACE build of the small-H kernels: stamps of wave 0 at j = 0..3, the
# other compute waves' pre-barrier stamps at j = 5..7 forward; backward j = 0..3 wave 0, 4 / 5
# the flush wave's step start / pre-barrier).  The stamps' own s_waitcnt lgkmcnt(0) serialises
# LDS traffic, so the traced step is slower than the untraced one; the split is what counts.
Tp = (T + 15) // 16 * 16


def small_traced(fn):
    buf = torch.zeros(B * 2 * Tp * 8, dtype=torch.int64, device=dev)
    _lib.call("avc_lstm_trace", buf.data_ptr())
    try:
        fn()
        torch.cuda.synchronize()
    finally:
        _lib.call("avc_lstm_trace", None)
    return buf.cpu().numpy().reshape(B * 2, Tp, 8).astype(np.float64) * 1e-2


s = slice(1, T - 1)
st = small_traced(lambda: K.lstm_fwd(xproj, whh, B, T, H, 2))
per = np.diff(st[:, :T, 0], axis=1)[:, 1:].mean()
dot = (st[:, s, 1] - st[:, s, 0]).mean()
cell = (st[:, s, 2] - st[:, s, 1]).mean()
wr = (st[:, s, 3] - st[:, s, 2]).mean()
last = np.maximum(st[:, s, 3], st[:, s, 5:8].max(axis=2))
bar = (st[:, 2:T, 0] - last).mean()
print(f"BiLSTM fwd traced: period {per:5.3f} | dot {dot:5.3f} cell {cell:5.3f} write {wr:5.3f} "
      f"last-wave -> next step {bar:5.3f} us", flush=True)
st = small_traced(lambda: K.lstm_bwd(dh, h, c, g, whh, None, B, T, H, 2))
per = np.diff(st[:, :T, 0], axis=1)[:, 1:].mean()
dot = (st[:, s, 1] - st[:, s, 0]).mean()
cell = (st[:, s, 2] - st[:, s, 1]).mean()
wr = (st[:, s, 3] - st[:, s, 2]).mean()
bar = (st[:, 2:T, 0] - np.maximum(st[:, s, 3], st[:, s, 5])).mean()
print(f"BiLSTM bwd traced: period {per:5.3f} | dot {dot:5.3f} cell {cell:5.3f} write {wr:5.3f} "
      f"last-wave -> next step {bar:5.3f} us", flush=True)
