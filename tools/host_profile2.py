"""Host enqueue of TrainStep.step (AutoVC C2) with the autograd engine's device thread on / off
(torch.autograd.set_multithreading_enabled), and a cProfile of the whole step with the backward on
the calling thread (so the profile sees the backward's Python too).  python tools/host_profile2.py"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
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
    for mt in (True, False, True, False):
        torch.autograd.set_multithreading_enabled(mt)
        for _ in range(3):
            ts.step(x, e)
        torch.cuda.synchronize()
        host = []
        t0 = time.perf_counter()
        for _ in range(20):
            h0 = time.perf_counter()
            ts.step(x, e)
            host.append(time.perf_counter() - h0)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        host.sort()
        print(f"multithreading {mt}: host enqueue median {host[10] * 1e3:.2f} ms; wall {(t2 - t0) / 20 * 1e3:.2f} ms/step",
              flush=True)
    torch.autograd.set_multithreading_enabled(False)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(10):
        ts.step(x, e)
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(45)


if __name__ == "__main__":
    main()
