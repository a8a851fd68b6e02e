"""BN backward at the C2 production shape and dtypes (M = 8192 frames, C = 512, bf16 dA / y,
bf16-only dy, ReLU from the recomputed pre-activation): per-call time by HIP events.
Run under rocprofv3 --kernel-trace --stats for the per-kernel split."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import autoformer_amd as A  # noqa: E402
from autoformer_amd import kernels as K  # noqa: E402

A.set_compute("bf16")
dev = "cuda:0"
M, C = (int(v) for v in sys.argv[1:3]) if len(sys.argv) > 2 else (8192, 512)
torch.manual_seed(0)
y = torch.randn(M, C, device=dev).to(torch.bfloat16)
dA = torch.randn(M, C, device=dev).to(torch.bfloat16)
mean = y.float().mean(0)
rstd = 1.0 / (y.float().var(0, unbiased=False) + 1e-5).sqrt()
g, b = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)


def bwd():
    return K.bn_bwd(dA, None, y, mean, rstd, g, K.ACT_RELU, beta=b, dy_bf16=True)


# fp64 reference of the same formulas
yh = (y.double() - mean.double()) * rstd.double()
z = yh * g.double() + b.double()
dz = dA.double() * (z > 0)
m1, m2 = dz.mean(0), (dz * yh).mean(0)
ref = g.double() * rstd.double() * (dz - m1 - yh * m2)
out, dgam, dbet, dbias = bwd()
err = (out.double() - ref).abs().max().item() / ref.abs().max().item()
print(f"rel-inf dy {err:.2e}  dgamma {((dgam.double() - (dz * yh).sum(0)).abs().max() / (dz * yh).sum(0).abs().max()).item():.2e}"
      f"  dbeta {((dbet.double() - dz.sum(0)).abs().max() / dz.sum(0).abs().max()).item():.2e}", flush=True)
for _ in range(5):
    bwd()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
n = 200
e0.record()
for _ in range(n):
    bwd()
e1.record()
torch.cuda.synchronize()
print(f"BN bwd M={M} C={C}: {e0.elapsed_time(e1) / n * 1000:.2f} us/call", flush=True)
