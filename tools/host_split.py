"""Host enqueue of one TrainStep.step (AutoVC C2) split into its phases -- forward + losses,
backward, optimizer / joins -- with no synchronisation inside the step, and a cProfile of the
backward and forward phases by cumulative time.   python tools/host_split.py [--steps 20]"""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--model", default="AutoVC")
    args = ap.parse_args()
    import importlib

    import autoformer_amd as A
    from autoformer_amd import train as TR
    from autoformer_amd.detinit import det_init_, det_inputs
    from autoformer_amd.layers import join_side

    A.set_compute("bf16")
    T, freq = (128, 16) if args.model == "AutoVC" else (176, 22)
    cls = getattr(importlib.import_module(f"autoformer_amd.factory.{args.model}"), args.model)
    m = cls(44, 256, 512, freq)
    det_init_(m)
    m = m.cuda().train()
    x, e = det_inputs(64, T)
    x, e = torch.from_numpy(x).cuda(), torch.from_numpy(e).cuda()
    ts = TR.TrainStep(m)
    for _ in range(3):
        ts.step(x, e)
    torch.cuda.synchronize()
    phases = {"zero+fwd+loss": [], "backward": [], "join+adam+prefetch": []}

    def one(prof=None):
        t0 = time.perf_counter()
        ts.gflat.zero_()
        ts.model._decoder_bwd_done = ts._decoder_done if ts.split is not None else None
        if prof is not None:
            prof.enable()
        loss, parts, x_psnt = ts.loss_fn(ts.model, x, e, ts.lambda_cd)
        t1 = time.perf_counter()
        loss.backward()
        t2 = time.perf_counter()
        if prof is not None:
            prof.disable()
        ts.model._decoder_bwd_done = None
        join_side()
        ts._finish()
        TR.prefetch_packs()
        t3 = time.perf_counter()
        return t1 - t0, t2 - t1, t3 - t2

    for _ in range(args.steps):
        a, b, c = one()
        phases["zero+fwd+loss"].append(a)
        phases["backward"].append(b)
        phases["join+adam+prefetch"].append(c)
        torch.cuda.synchronize()
    for k, v in phases.items():
        v = sorted(v)
        print(f"{k:20s} median {v[len(v) // 2] * 1e3:6.2f} ms  min {v[0] * 1e3:6.2f} ms")
    torch.autograd.set_multithreading_enabled(False)  # the backward's Python on this thread for the profile
    pr = cProfile.Profile()
    for _ in range(5):
        one(pr)
        torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
