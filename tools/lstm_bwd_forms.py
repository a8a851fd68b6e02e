"""A/B of the persistent backward recurrence forms at the AutoVC decoder shapes (B=64, T=128):
event time per launch (the sentinel forms include their twin fill), the in-kernel per-step
timeline (avc_lstm_trace stamps, as tools/lstm_trace.py), and the output difference against the
flag-gather form.

  python tools/lstm_bwd_forms.py [reps]

Forms: 0 flag gather, 2 sentinel hand-off, 3 sentinel + XCD-verified L2-resident stores."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import autoformer_amd as A  # noqa: E402
from autoformer_amd import kernels as K  # noqa: E402

from autoformer_amd import _lib  # noqa: E402

A.set_compute("bf16")
dev = "cuda:0"
B, T = 64, 128
REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 3
FORMS = [int(f) for f in os.environ.get("FORMS", "0,2,3").split(",")]
HS = [int(f) for f in os.environ.get("HS", "1024,512").split(",")]


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
    """wait = step start -> exchange complete, prod -> product reduced, tail -> published;
    handoff = consumer's exchange complete - the LAST publish of its group's previous step."""
    nwg = st.shape[0]
    s = slice(1, T)
    wait = (st[:, s, 1] - st[:, s, 0]).mean()
    prod = (st[:, s, 2] - st[:, s, 1]).mean()
    tail = (st[:, s, 3] - st[:, s, 2]).mean()
    period = np.diff(st[:, :, 0], axis=1)[:, 1:].mean()
    hand = []
    for g in range(ng):
        mem = [b for b in range(nwg) if b % ng == g]
        last_pub = st[mem, :-1, 3].max(axis=0)
        ready = st[mem, 1:, 1]
        hand.append((ready - last_pub[None, :]).mean())
    skew = (st[:, s, 3].max(axis=0) - st[:, s, 3].min(axis=0)).mean()
    span = st[:, -1, 3].max() - st[:, 0, 0].min()
    print(f"{tag}: span {span:8.1f} us = {span / T:5.2f} us/step | wait {wait:5.2f} prod {prod:5.2f} "
          f"tail {tail:5.2f} period {period:5.2f} handoff {np.mean(hand):5.2f} publish-skew {skew:5.2f}",
          flush=True)


def ev_time(fn, n=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


for H in HS:
    G = 4 * H
    torch.manual_seed(0)
    xproj = torch.randn(B * T, G, device=dev) * 0.1
    whh = (torch.randn(G, H, device=dev) * 0.02).bfloat16()
    whht = whh.t().contiguous()
    hbuf = K.lstm_scratch(B, H, 1, dev)
    h, c, g = K.lstm_fwd(xproj, whh, B, T, H, 1, hbuf)
    dh = torch.randn_like(h) * 0.1
    gbuf = K.lstm_bwd_scratch(B, H, 1, dev)
    ng = (B + 7) // 8
    nwg = ng * (H // 32)
    ref = None
    res = {}
    for rep in range(REPS):
        for form in FORMS:
            K.lstm_set_bwd_form(form)
            run = lambda: K.lstm_bwd(dh, h, c, g, None, whht, B, T, H, 1, gbuf=gbuf)  # noqa: E731
            us = ev_time(run)
            res.setdefault(form, []).append(us)
            if rep == 0:
                out = run()
                torch.cuda.synchronize()
                assert K.lstm_bwd_timeout_flag(gbuf, B, H) == 0
                if ref is None:
                    ref = out.clone()
                d = ((out - ref).norm() / ref.norm()).item()
                tw = (out._bf16.float() - out.to(torch.bfloat16).float()).abs().max().item()
                print(f"H={H} form {form}: {us:8.1f} us/launch ({us / T:5.2f} us/step)  rel-frob vs form 0 {d:.2e}"
                      f"  twin max|diff| {tw:.1e}", flush=True)
                report(f"H={H} form {form}", traced(run, nwg), ng)
    for form, v in res.items():
        print(f"H={H} form {form}: median {np.median(v):8.1f} us  all {' '.join(f'{x:.1f}' for x in v)}", flush=True)
K.lstm_set_bwd_form(-1)
