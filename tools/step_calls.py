"""The recorded C2 step (TrainStep.record) as a list: every native call in order with its stream and,
for the event plumbing (avc_event_record / avc_stream_wait_event), the event handle -- the stream
edges of the step -- plus the model-side call site.  Finds what a main-queue gap in a kernel trace is
waiting for.

  python tools/step_calls.py [--model AutoVC] [--disc] > calls.txt
"""
import argparse
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="AutoVC")
    args = ap.parse_args()
    import importlib

    import autoformer_amd as A
    from autoformer_amd import _lib
    from autoformer_amd.detinit import det_init_, det_inputs
    from autoformer_amd.train import TrainStep

    A.set_compute("bf16")
    T, freq = (128, 16) if args.model == "AutoVC" else (176, 22)
    m = getattr(importlib.import_module(f"autoformer_amd.factory.{args.model}"), args.model)(44, 256, 512, freq)
    det_init_(m)
    m = m.cuda().train()
    x, e = det_inputs(64, T)
    x, e = torch.from_numpy(x).cuda(), torch.from_numpy(e).cuda()
    ts = TrainStep(m)
    ts.step(x, e)
    torch.cuda.synchronize()
    streams = {}
    sites = []
    real = _lib.call
    pkg = os.path.join("autoformer_amd", "")

    def rec(name, *a):
        site = "?"
        for fr in reversed(traceback.extract_stack()[:-1]):
            if pkg in fr.filename and not fr.filename.endswith(("kernels.py", "_lib.py", "replay.py")):
                site = fr.filename.split(pkg)[-1] + f":{fr.lineno}"
                break
        sites.append(site)
        return real(name, *a)

    _lib.call = rec
    try:
        rec_ = ts.record(x, e, warmup=0)
    finally:
        _lib.call = real
    names = {int(torch.cuda.current_stream().cuda_stream): "main"}
    i = 0
    for fn, name, a in rec_.calls:
        if fn is None:
            print(f"{'':5s} <marker>")
            continue
        site = sites[i] if i < len(sites) else "?"
        i += 1
        if name in ("avc_event_record", "avc_stream_wait_event"):
            ev, st = (a[0], a[1]) if name == "avc_event_record" else (a[1], a[0])
            st = int(st or 0)
            sname = names.setdefault(st, f"s{len(names)}")
            print(f"{i:5d} {sname:5s} {name:24s} ev={int(ev or 0):#x}  {site}")
            continue
        st = a[-1] if a and isinstance(a[-1], int) else None
        sname = names.setdefault(int(st), f"s{len(names)}") if st else "-"
        print(f"{i:5d} {sname:5s} {name:24s} {site}")


if __name__ == "__main__":
    main()
