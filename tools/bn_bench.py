"""Per-call time of the train-mode BN forward (stats merge + apply) and backward at the C2 shape
(M = 8192 frames, C = 512 channels); AVC_BN_FUSED=0 selects the separate finalize launches."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import autoformer_amd as A  # noqa: E402
from autoformer_amd import kernels as K  # noqa: E402

A.set_compute("bf16")
dev = "cuda:0"
M, C = 8192, 512
x = torch.randn(M, 512, device=dev)
w = torch.randn(C, 512, device=dev)
y = torch.empty(M, C, device=dev)
part = K.bn_partial_buffer(M, C, dev)
K.gemm(M, C, 512, K.operand(x, 512), K.operand(w, 512), y, bn_partial=part)
g, b = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
dA = torch.randn(M, C, device=dev)


def fwd():
    return K.bn_apply_stats(y, part, g, b, rm, rv, None, 0.1, 1e-5, K.ACT_RELU)


a, (mean, rstd, _, _) = fwd()


def bwd():
    return K.bn_bwd(dA, None, y, mean, rstd, g, K.ACT_RELU, beta=b)


for name, fn in (("fwd", fwd), ("bwd", bwd)):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    n = 200
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"BN {name} fused={os.environ.get('AVC_BN_FUSED', '1')}: {e0.elapsed_time(e1) / n * 1000:.2f} us/call",
          flush=True)
