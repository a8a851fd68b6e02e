"""Forward-graph diagnostic, part 2: after replay -> eager backward -> replay, which tensors saved
by the retained autograd graph hold non-finite values, listed from the graph's inputs outwards
(the first one is the forward op that read memory the eager backward had changed).
python tools/graph_fwd_probe2.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def nodes_of(loss):
    order, seen, stack = [], set(), [(loss.grad_fn, 0)]
    while stack:
        n, d = stack.pop()
        if n is None or n in seen:
            continue
        seen.add(n)
        order.append((d, n))
        for nxt, _ in n.next_functions:
            stack.append((nxt, d + 1))
    return order


def saved(n):
    out = []
    try:
        ts = n.saved_tensors
    except Exception:
        ts = ()
    for t in ts:
        if isinstance(t, torch.Tensor):
            out.append(t)
    for k in dir(n):
        if k.startswith("_") or k in ("saved_tensors", "next_functions", "metadata", "needs_input_grad"):
            continue
        try:
            v = getattr(n, k)
        except Exception:
            continue
        if isinstance(v, torch.Tensor):
            out.append(v)
        elif isinstance(v, (tuple, list)):
            out += [t for t in v if isinstance(t, torch.Tensor)]
    return out


def main():
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
        ts.graph_f.replay()
        torch.cuda.synchronize()
        order = nodes_of(ts.loss)
        ref = {}
        for d, n in order:
            for i, t in enumerate(saved(n)):
                ref[(id(n), i)] = t.detach().clone()
        ts.gflat.zero_()
        ts.loss.backward(retain_graph=True)
        join_side()
        torch.cuda.synchronize()
        # which saved tensors did the backward itself change?
        for d, n in sorted(order, key=lambda p: -p[0]):
            for i, t in enumerate(saved(n)):
                r = ref[(id(n), i)]
                if t.shape == r.shape and not torch.equal(t.detach(), r):
                    print(f"after backward: depth {d} {type(n).__name__} saved[{i}] {tuple(t.shape)} {t.dtype} changed",
                          flush=True)
        ts.graph_f.replay()
        torch.cuda.synchronize()
        print("loss after second replay", ts.loss.item())
        for d, n in sorted(order, key=lambda p: -p[0]):
            for i, t in enumerate(saved(n)):
                tf = t.detach().float()
                r = ref[(id(n), i)].float()
                bad = not torch.isfinite(tf).all().item()
                diff = (tf - r).abs().max().item() if tf.shape == r.shape and torch.isfinite(tf).all() else float("nan")
                if bad or diff > 0:
                    print(f"after replay 2: depth {d} {type(n).__name__} saved[{i}] {tuple(t.shape)} nonfinite={bad} "
                          f"maxdiff={diff:.3e}", flush=True)
    finally:
        set_grad_sink(False)


if __name__ == "__main__":
    main()
