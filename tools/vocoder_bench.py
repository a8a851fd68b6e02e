"""MelGAN generator (melgan/modules.py:88-131) on the HIP path: latency of one conversion-sized
utterance (B=1, T=176 mel frames -> 45,056 samples) and throughput at B=16, bf16 compute,
closed-form weights.  Algorithmic FLOP per mel frame counted from the layer shapes
(polyphase ConvTranspose counted at its true 2 taps, not the 3-tap window the GEMM runs)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import autoformer_amd as A  # noqa: E402
from autoformer_amd.detinit import det_mel, det_melgan_state  # noqa: E402
from autoformer_amd.melgan import Generator  # noqa: E402

A.set_compute(os.environ.get("AUTOVC_COMPUTE", "bf16"))
g = Generator(80, 32, 3)
g.load_state_dict({k: torch.from_numpy(v) for k, v in
                   det_melgan_state([(k, tuple(v.shape)) for k, v in g.state_dict().items()]).items()})
g = g.to("cuda:0")


def flop_per_frame(ngf=32, nres=3, C_in=80):
    f, rate, C = 2 * C_in * 16 * ngf * 7, 1, 16 * ngf
    for r in (8, 8, 2, 2):
        f += 2 * C * (C // 2) * 2 * rate * r     # ConvTranspose: 2 taps per output sample
        rate, C = rate * r, C // 2
        f += nres * rate * 2 * (C * C * 3 + C * C + C * C)
    return f + rate * 2 * C * 7


def timed(B, T, reps):
    mel = torch.from_numpy(det_mel(B, 80, T)).cuda()
    for _ in range(3):
        g(mel)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g(mel)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


fpf = flop_per_frame()
res = {"flop_per_mel_frame": fpf}
for B, T, reps in ((1, 176, 50), (16, 176, 20)):
    ms = timed(B, T, reps)
    res[f"B{B}_T{T}"] = {"ms": round(ms, 3), "samples_per_s": round(B * T * 256 / ms * 1e3),
                          "tflops": round(B * T * fpf / ms * 1e-9, 2)}
print(json.dumps(res))
