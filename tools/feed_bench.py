"""Train step fed from disk through autoformer_amd.data (get_loader + DeviceFeed) vs the same
step on a batch resident in HBM: the host loading / pinned H2D path must stay hidden.

  python tools/feed_bench.py [--steps 20]   (writes a synthetic VCTK-layout dataset under /tmp)
"""
import argparse
import os
import pickle
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def make_dataset(root, speakers=109, utts=4, seed=0):  # VCTK: 109 speakers
    rng = np.random.RandomState(seed)
    meta = []
    for s in range(speakers):
        spk = f"p{s:03d}"
        os.makedirs(os.path.join(root, spk), exist_ok=True)
        emb = rng.randn(256).astype(np.float32)
        emb /= np.linalg.norm(emb)
        entry = [spk, emb]
        for u in range(utts):
            T = int(rng.randint(100, 400))
            np.save(os.path.join(root, spk, f"{u}.npy"), (rng.rand(T, 80) * 7 - 5).astype(np.float32))
            entry.append(f"{spk}/{u}.npy")
        meta.append(entry)
    with open(os.path.join(root, "train.pkl"), "wb") as f:
        pickle.dump(meta, f)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    import autoformer_amd as A
    from autoformer_amd.data import DeviceFeed, get_loader
    from autoformer_amd.detinit import det_init_
    from autoformer_amd.factory.AutoVC import AutoVC
    from autoformer_amd.train import TrainStep

    A.set_compute("bf16")
    root = tempfile.mkdtemp(prefix="vctk_", dir="/tmp")
    t0 = time.perf_counter()
    make_dataset(root)
    loader = get_loader(root, batch_size=64, len_crop=128)
    print(f"dataset: {len(loader.dataset)} speakers loaded in {time.perf_counter() - t0:.2f} s", flush=True)
    m = AutoVC(44, 256, 512, 16)
    det_init_(m)
    m = m.cuda().train()
    ts = TrainStep(m)

    it = iter(DeviceFeed(loader, "cuda:0", repeat=True))
    x, e = next(it)
    for _ in range(3):
        ts.step(x, e)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        x, e = next(it)
        ts.step(x, e)
    torch.cuda.synchronize()
    fed = (time.perf_counter() - t0) / args.steps
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ts.step(x, e)
    torch.cuda.synchronize()
    res = (time.perf_counter() - t0) / args.steps
    print(f"fed from disk via DeviceFeed: {fed * 1e3:.3f} ms/step ({64 * 128 / fed:.0f} frames/s); "
          f"resident batch: {res * 1e3:.3f} ms/step ({64 * 128 / res:.0f} frames/s)")


if __name__ == "__main__":
    main()
