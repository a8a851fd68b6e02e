"""In-kernel timeline of the encoder BiLSTM recurrences (lstm_small_fwd / _bwd TRACE builds,
avc_lstm_trace): per step, wave 0 stamps step start (0), product done (1), cell update done
(2), before the barrier (3); the flush wave stamps its step start (4) and pre-barrier (5).
Prints the mean per-step phases (us) over all workgroups."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import autoformer_amd as A  # noqa: E402
from autoformer_amd import _lib as L  # noqa: E402
from autoformer_amd import kernels as K  # noqa: E402

dev = "cuda:0"
A.set_compute(os.environ.get("MODE", "bf16"))
B, H, T = 64, 44, 128
nblk = 2 * B


def traced(fn):
    buf = torch.zeros(nblk * T * 8, dtype=torch.int64, device=dev)
    L.call("avc_lstm_trace", buf.data_ptr())
    try:
        fn()
        torch.cuda.synchronize()
    finally:
        L.call("avc_lstm_trace", None)
    st = buf.view(nblk, T, 8).cpu().numpy().astype(np.float64) / 100.0  # us
    return st


def report_fwd_waves(st):
    """Forward build: j = 3, 5, 6, 7 are the four compute waves' pre-barrier stamps."""
    pre = st[:, :, [3, 5, 6, 7]]
    spread = (pre.max(axis=2) - pre.min(axis=2)).mean()
    late = np.bincount(pre.argmax(axis=2).ravel(), minlength=4)
    after = (st[:, 1:, 0] - pre[:, :-1].max(axis=2)).mean()
    per_i = [(st[:, i + 1::16, 0][:, :7] - st[:, i:-1:16, 0][:, :7]).mean() for i in range(15)]
    print(f"fwd waves: pre-barrier spread {spread:.3f} us, last-arriving wave counts {late.tolist()}, "
          f"last arrival -> next step start {after:.3f} us; period by step-in-chunk "
          + " ".join(f"{v:.2f}" for v in per_i), flush=True)


def report(tag, st):
    prod = (st[:, :, 1] - st[:, :, 0]).mean()
    cell = (st[:, :, 2] - st[:, :, 1]).mean()
    tail = (st[:, :, 3] - st[:, :, 2]).mean()
    bar = (st[:, 1:, 0] - st[:, :-1, 3]).mean()
    period = (st[:, 1:, 0] - st[:, :-1, 0]).mean()
    chunk0 = (st[:, 16::16, 0] - st[:, 15:-1:16, 0]).mean()
    flush = (st[:, 16::16, 5] - st[:, 16::16, 4]).mean()
    other = (st[:, 1:, 5] - st[:, 1:, 4])
    print(f"{tag}: period {period:.3f} us/step | product {prod:.3f} cell {cell:.3f} tail {tail:.3f} "
          f"barrier {bar:.3f} | chunk-boundary step {chunk0:.3f} (flush {flush:.3f}), flush-wave step "
          f"median {np.median(other):.3f}", flush=True)


G = 4 * H
xproj = torch.randn(B * T, 2 * G, device=dev) * 0.5
whh = torch.randn(2 * G, H, device=dev) * 0.1
K.lstm_fwd(xproj, whh, B, T, H, 2)
stf = traced(lambda: K.lstm_fwd(xproj, whh, B, T, H, 2))
report("fwd", stf)
report_fwd_waves(stf)
h, c, g = K.lstm_fwd(xproj, whh, B, T, H, 2)
dh = torch.randn_like(h)
report("bwd", traced(lambda: K.lstm_bwd(dh, h, c, g, whh, None, B, T, H, 2)))
