"""LSTM recurrence microbenchmark: per-launch time of the step kernels (events), plus the
floor with no recurrent product (T=1 launches only run the s=0 path)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import autoformer_amd as A
from autoformer_amd import kernels as K

A.set_compute("bf16")
dev = "cuda:0"


def ev_time(fn, reps=5):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for (B, H, T) in [(64, 1024, 128), (64, 512, 128), (64, 1024, 1)]:
    G = 4 * H
    xproj = torch.randn(B * T, G, device=dev) * 0.1
    whh = (torch.randn(G, H, device=dev) * 0.02).bfloat16()
    whht = whh.t().contiguous()
    hbuf = K.lstm_scratch(B, H, 1, dev)
    us = ev_time(lambda: K.lstm_fwd(xproj, whh, B, T, H, 1, hbuf))
    h, c, g = K.lstm_fwd(xproj, whh, B, T, H, 1, hbuf)
    dh = torch.randn_like(h)
    usb = ev_time(lambda: K.lstm_bwd(dh, h, c, g, None, whht, B, T, H, 1))
    print(f"B={B} H={H} T={T}: fwd {us/T:7.2f} us/step  bwd {usb/T:7.2f} us/step", flush=True)
