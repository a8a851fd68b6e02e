"""Diagnostic of the forward-only hipGraph (TrainStep.capture(forward_only=True)) at C2: which
step of the eager part between two replays makes the second replay's loss differ from the eager
step's.  Variants: replay twice with nothing between / after an eager backward / after the
backward + Adam / after backward + Adam + pack prefetch.   python tools/graph_fwd_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def run(variant):
    import autoformer_amd as A
    from autoformer_amd import train as TR
    from autoformer_amd.detinit import det_init_, det_inputs
    from autoformer_amd.factory.AutoVC import AutoVC
    from autoformer_amd.layers import join_side, set_grad_sink

    A.set_compute("bf16")
    m = AutoVC(44, 256, 512, 16)
    det_init_(m)
    m = m.cuda().train()
    x, e = det_inputs(64, 128)
    x, e = torch.from_numpy(x).cuda(), torch.from_numpy(e).cuda()
    ts = TR.TrainStep(m, lr=0.0)
    try:
        ts.step(x, e)
        ts.capture(x, e, warmup=0, forward_only=True)
        out = []
        for i in range(3):
            ts.graph_f.replay()
            torch.cuda.synchronize()
            out.append(ts.loss.item())
            if variant >= 1:
                ts.gflat.zero_()
                ts.loss.backward(retain_graph=True)
                join_side()
            if variant >= 2:
                ts._finish()
            if variant >= 3:
                TR.prefetch_packs()
            torch.cuda.synchronize()
        fault = ""
        try:
            ts.check()
        except Exception as ex:  # noqa: BLE001
            fault = f" FAULT {type(ex).__name__}: {ex}"
        print(f"variant {variant}: losses {out}{fault}", flush=True)
    finally:
        set_grad_sink(False)


if __name__ == "__main__":
    for v in (map(int, sys.argv[1].split(",")) if len(sys.argv) > 1 else (0, 1, 2, 3)):
        run(v)
