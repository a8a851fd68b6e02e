"""Latency of one AutoVC conversion (B=1 utterance, forward only, bf16 compute) through
autoformer_amd.convert.Converter, host mel in -> host mel out.

  python tools/convert_bench.py [--len-crop 176] [--reps 50]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--len-crop", type=int, default=176)
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    import autoformer_amd as A
    from autoformer_amd.convert import Converter
    from autoformer_amd.detinit import det_init_, det_inputs
    from autoformer_amd.factory.AutoVC import AutoVC

    A.set_compute("bf16")
    T = args.len_crop
    freq = 22 if T % 22 == 0 else 16
    m = AutoVC(44, 256, 512, freq)
    det_init_(m)
    m = m.cuda().train()
    x, e = det_inputs(2, T)
    conv = Converter(m, T)
    for _ in range(5):
        conv.convert(x[0], e[0], e[1])
    torch.cuda.synchronize()
    ts = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        conv.convert(x[0], e[0], e[1])
        ts.append(time.perf_counter() - t0)
    ts.sort()
    print(f"conversion B=1 T={T}: median {ts[len(ts) // 2] * 1e3:.2f} ms, min {ts[0] * 1e3:.2f} ms "
          f"(host mel in -> host mel out, {T * 80 * 4 / 1e3:.0f} KB each way)")


if __name__ == "__main__":
    main()
