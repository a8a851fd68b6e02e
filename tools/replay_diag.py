"""Replay vs eager loss trace (tests/test_gpu_replay.py's C2 comparison, printed per step) under the
current environment; mode "interleaved" steps both trainers alternately, "sequential" runs the eager
trainer's steps first.  python tools/replay_diag.py [interleaved|sequential] [steps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "interleaved"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    import autoformer_amd as A
    import autoformer_amd.kernels as K
    from autoformer_amd.detinit import det_init_, det_inputs
    from autoformer_amd.train import TrainStep
    from factory.AutoVC import AutoVC

    A.set_compute("bf16")
    K.set_deterministic(True)
    dev = "cuda:0"

    def make():
        m = AutoVC(44, 256, 512, 16)
        det_init_(m)
        m = m.to(dev).train()
        return m, TrainStep(m, lr=1e-4)

    batches = [tuple(torch.from_numpy(a).to(dev) for a in det_inputs(64, 128, seed=40 + i)) for i in range(steps)]
    (ma, ta), (mb, tb) = make(), make()
    la_all = []
    if mode == "sequential":
        for i, (x, e) in enumerate(batches):
            la_all.append(ta.step(x, e).item())
    xb, eb = batches[1][0].clone(), batches[1][1].clone()
    tb.step(*batches[0])
    for i, (x, e) in enumerate(batches):
        if mode == "interleaved":
            la_all.append(ta.step(x, e).item())
        if i == 0:
            lb = None
        elif i == 1:
            tb.record(xb, eb, warmup=0)
            lb = tb.loss.item()
        else:
            lb = tb.step(x, e).item()
        torch.cuda.synchronize()
        print(f"step {i}: eager {la_all[i]:.6f} replay {lb}", flush=True)
    tb.check()


if __name__ == "__main__":
    main()
