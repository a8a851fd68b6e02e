"""Replay-vs-eager check of TrainStep.capture at C2 (B=64, T=128, bf16), lr = 0, a new batch per
replay: prints per replay the loss of both and the worst gradient deviation.  Debug knobs of
graph.hip via the environment (AVC_GRAPH_SPLIT, AVC_GRAPH_SERIAL, AVC_GRAPH_CLONE_ONLY).
  python tools/graph_check.py [steps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    import autoformer_amd as A
    from autoformer_amd.detinit import det_init_, det_inputs
    from autoformer_amd.factory.AutoVC import AutoVC
    from autoformer_amd.train import TrainStep

    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    B, T = 64, 128
    A.set_compute("bf16")
    dev = "cuda:0"

    def model():
        m = AutoVC(44, 256, 512, 16)
        det_init_(m)
        return m.to(dev).train()

    batches = [tuple(torch.from_numpy(a).to(dev) for a in det_inputs(B, T, seed=20 + i)) for i in range(steps)]
    ma, mb = model(), model()
    ta, tb = TrainStep(ma, lr=0.0), TrainStep(mb, lr=0.0)
    xb, eb = batches[0][0].clone(), batches[0][1].clone()
    tb.step(xb, eb)
    tb.capture(xb, eb, warmup=0)
    print("split:", None if tb.graph_split is None else tb.graph_split.counts, flush=True)
    from autoformer_amd import kernels as K
    for i, (x, e) in enumerate(batches):
        pre = [n for n, p in mb.named_parameters() if not torch.isfinite(p).all()]
        st = tb.opt.state.tolist()
        mv = bool(torch.isfinite(tb.opt.m).all() and torch.isfinite(tb.opt.v).all())
        print(f"before replay {i}: non-finite params {len(pre)}, adam state {st}, m/v finite {mv}, "
              f"fault word {int(K.fault_word().item())}", flush=True)
        la = ta.step(x, e)
        xb.copy_(x)
        eb.copy_(e)
        lb = tb.step(xb, eb)
        torch.cuda.synchronize()
        worst, wn = 0.0, ""
        nan = []
        for (n, pa), (_, pb) in zip(ma.named_parameters(), mb.named_parameters()):
            a, b = pa.grad.double(), pb.grad.double()
            if not torch.isfinite(b).all():
                nan.append(n)
                continue
            d = ((a - b).norm() / a.norm().clamp_min(1e-12)).item()
            if d > worst:
                worst, wn = d, n
        pn = [n for n, p in mb.named_parameters() if not torch.isfinite(p).all()]
        print(f"replay {i}: loss eager {la.item():.6f} graph {lb.item():.6f}; worst grad dev {worst:.2e} ({wn}); "
              f"non-finite grads {nan[:4]} ({len(nan)}); non-finite params {pn[:4]} ({len(pn)})", flush=True)
    tb.check()


if __name__ == "__main__":
    main()
