"""How long the main stream waits at the end of the backward for the side stream (weight
gradients) -- events recorded on the main stream just before and just after join_side().

  python tools/tail_time.py [--steps 20]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    import autoformer_amd as A
    from autoformer_amd import layers as Lyr
    from autoformer_amd import train as Tr
    from autoformer_amd.detinit import det_init_, det_inputs
    from autoformer_amd.factory.AutoVC import AutoVC

    A.set_compute("bf16")
    m = AutoVC(44, 256, 512, 16)
    det_init_(m)
    m = m.cuda().train()
    x, e = det_inputs(64, 128)
    x, e = torch.from_numpy(x).cuda(), torch.from_numpy(e).cuda()
    ts = Tr.TrainStep(m)
    evs = []
    real = Lyr.join_side

    def timed_join():
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        real()
        b.record()
        evs.append((a, b))

    Tr.join_side = timed_join
    for _ in range(3):
        ts.step(x, e)
    torch.cuda.synchronize()
    evs.clear()
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0.record()
    for _ in range(20):
        ts.step(x, e)
    s1.record()
    torch.cuda.synchronize()
    waits = sorted(a.elapsed_time(b) * 1e3 for a, b in evs)
    print(f"step {s0.elapsed_time(s1) / 20:.3f} ms; end-of-backward wait for the side stream: "
          f"median {waits[len(waits) // 2]:.1f} us, min {waits[0]:.1f}, max {waits[-1]:.1f}")


if __name__ == "__main__":
    main()
