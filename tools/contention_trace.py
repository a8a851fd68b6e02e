"""Driver for a kernel trace of the recorded C2 step, WITHOUT bench.py's refusal of diagnostic
ablations: run it under rocprofv3 once as is and once with AVC_ABLATE_WGRAD=1 (no weight-gradient
side stream: wrong gradients, diagnostic only), then tools/contention_diff.py pairs the main-queue
kernels of the two traces instance by instance (the inflation each one takes from the side stream).

  rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/contention_trace.py [steps]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench import synthetic_batch  # noqa: E402
from autoformer_amd import set_compute  # noqa: E402
from autoformer_amd.detinit import det_init_  # noqa: E402
from autoformer_amd.factory.AutoVC import AutoVC  # noqa: E402
from autoformer_amd.train import TrainStep  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dev = torch.device("cuda", 0)
    set_compute("bf16")
    model = AutoVC(44, 256, 512, 16)
    det_init_(model)
    model = model.to(dev).train()
    x, e = synthetic_batch(64, 128, 0, dev)
    tr = TrainStep(model, lr=1e-4)
    for _ in range(3):
        tr.step(x, e)
    tr.record(x, e, warmup=0)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(steps):
        tr.step(x, e)
    ev1.record()
    torch.cuda.synchronize()
    print(f"ablate_wgrad={os.environ.get('AVC_ABLATE_WGRAD', '0')} {ev0.elapsed_time(ev1) / steps:.4f} ms/step", flush=True)


if __name__ == "__main__":
    main()
