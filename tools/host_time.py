"""Host-side enqueue time of one TrainStep (no synchronisation inside the step) vs the GPU
step time: when the host takes longer than the GPU to queue a step, the GPU idles.

  python tools/host_time.py [--steps 20]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--replay", action="store_true", help="TrainStep.record + replayed steps")
    args = ap.parse_args()
    import autoformer_amd as A
    from autoformer_amd.detinit import det_init_, det_inputs
    from autoformer_amd.factory.AutoVC import AutoVC
    from autoformer_amd.train import TrainStep

    A.set_compute("bf16")
    m = AutoVC(44, 256, 512, 16)
    det_init_(m)
    m = m.cuda().train()
    x, e = det_inputs(64, 128)
    x, e = torch.from_numpy(x).cuda(), torch.from_numpy(e).cuda()
    ts = TrainStep(m)
    for _ in range(3):
        ts.step(x, e)
    if args.replay:
        rec = ts.record(x, e, warmup=0)
        print(f"recorded: {rec.native_calls()} native calls, torch ops {rec.torch_ops}")
        ts.step(x, e)
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        h0 = time.perf_counter()
        ts.step(x, e)
        host.append(time.perf_counter() - h0)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    host.sort()
    print(f"host enqueue per step: median {host[len(host) // 2] * 1e3:.2f} ms, min {host[0] * 1e3:.2f} ms; "
          f"loop {(t1 - t0) / args.steps * 1e3:.2f} ms/step, drained after {(t2 - t1) * 1e3:.2f} ms; "
          f"wall {(t2 - t0) / args.steps * 1e3:.2f} ms/step")


if __name__ == "__main__":
    main()
