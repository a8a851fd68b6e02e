"""Encoder BiLSTM recurrences at the bench shape (B=64, T=128, H=44, 2 directions, bf16): launch
times with HIP events (isolated, 20 launches) and, for the MFMA kernels (lstm_mfma_fwd / _bwd), the
in-kernel per-step phases from their TRACE build (wave 0 stamps step start (0), product done (1),
cell update done (2)).  Run once per form:

  python tools/bilstm_trace.py                    # MFMA form (default)
  AVC_BILSTM_MFMA=0 python tools/bilstm_trace.py  # packed-FMA form (the default in the library)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import autoformer_amd as A  # noqa: E402
from autoformer_amd import _lib as L  # noqa: E402
from autoformer_amd import kernels as K  # noqa: E402

dev = "cuda:0"
A.set_compute("bf16")
B, H, T = 64, 44, 128
L.lib().avc_lstm_set_small_mfma(0 if os.environ.get("AVC_BILSTM_MFMA") == "0" else 1)
mfma = bool(L.lib().avc_lstm_small_mfma(H, K.BF16))
nblk = 2 * ((B + 3) // 4) if mfma else 2 * B


def timed(fn, n=20):
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) * 1e3 for a, b in ev]))


def traced(fn):
    buf = torch.zeros(nblk * T * 8, dtype=torch.int64, device=dev)
    L.call("avc_lstm_trace", buf.data_ptr())
    try:
        fn()
        torch.cuda.synchronize()
    finally:
        L.call("avc_lstm_trace", None)
    return buf.view(nblk, T, 8).cpu().numpy().astype(np.float64) / 100.0  # us


G = 4 * H
xproj = torch.randn(B * T, 2 * G, device=dev) * 0.5
whh = torch.randn(2 * G, H, device=dev) * 0.1
h, c, g = K.lstm_fwd(xproj, whh, B, T, H, 2)
dh = torch.randn_like(h)
fwd = lambda: K.lstm_fwd(xproj, whh, B, T, H, 2)  # noqa: E731
bwd = lambda: K.lstm_bwd(dh, h, c, g, whh, None, B, T, H, 2)  # noqa: E731
tf, tb = timed(fwd), timed(bwd)
print(f"{'mfma' if mfma else 'fma'} BiLSTM H={H} B={B} T={T}: fwd {tf:.1f} us ({tf / T:.3f}/step)  "
      f"bwd {tb:.1f} us ({tb / T:.3f}/step)  per C2 step (4 + 4 launches) {4 * (tf + tb):.0f} us", flush=True)
if mfma:
    for tag, fn in (("fwd", fwd), ("bwd", bwd)):
        st = traced(fn)
        prod = (st[:, :, 1] - st[:, :, 0]).mean()
        cell = (st[:, :, 2] - st[:, :, 1]).mean()
        rest = (st[:, 1:, 0] - st[:, :-1, 2]).mean()
        period = (st[:, 1:, 0] - st[:, :-1, 0]).mean()
        print(f"  {tag} traced: period {period:.3f} us/step | product {prod:.3f} cell {cell:.3f} "
              f"write+barrier {rest:.3f}", flush=True)
