"""cProfile of the host side of TrainStep.step (AutoVC C2): where the ~7 ms of Python per
step goes.   python tools/host_profile.py"""
import cProfile
import os
import pstats
import sys

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
    for _ in range(3):
        ts.step(x, e)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(10):
        ts.step(x, e)
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)
    st.sort_stats("cumtime").print_stats(35)


if __name__ == "__main__":
    main()
