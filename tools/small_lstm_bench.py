"""Encoder BiLSTM recurrence microbenchmark (H=44, 2 directions, B=64, T=128; the shape of
AutoVC.py:43,55): per-launch time of lstm_small_fwd / lstm_small_bwd (HIP events), bf16 and fp32
compute modes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import autoformer_amd as A  # noqa: E402
from autoformer_amd import kernels as K  # noqa: E402

dev = "cuda:0"


def ev_time(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for mode in ("bf16", "fp32"):
    A.set_compute(mode)
    for (B, H, T) in [(64, 44, 128), (64, 44, 176)]:
        G = 4 * H
        xproj = torch.randn(B * T, 2 * G, device=dev) * 0.5
        whh = torch.randn(2 * G, H, device=dev) * 0.1
        us = ev_time(lambda: K.lstm_fwd(xproj, whh, B, T, H, 2))
        h, c, g = K.lstm_fwd(xproj, whh, B, T, H, 2)
        dh = torch.randn_like(h)
        usb = ev_time(lambda: K.lstm_bwd(dh, h, c, g, whh, None, B, T, H, 2))
        print(f"{mode} B={B} H={H} T={T} dirs=2: fwd {us:7.1f} us ({us / T:5.3f} us/step)  "
              f"bwd {usb:7.1f} us ({usb / T:5.3f} us/step)", flush=True)
