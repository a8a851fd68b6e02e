"""Fixtures for the training-data path, produced by the REFERENCE loader itself
(/root/reference/util/data_loader.py:20-102, imported read-only in this container with
PYTHONDONTWRITEBYTECODE=1; the reference never ships with this repo).

The dataset is a miniature tree in the reference layout, generated deterministically by
`build_tree` (tests/test_data.py rebuilds the identical tree): 5 speakers, 2-4 utterances each,
lengths shorter than / equal to / longer than len_crop, one path with a backslash.  Recorded:
  * items: np.random.seed(1234), then dataset[i] for a fixed index sequence (Utterances.__getitem__,
    data_loader.py:63-81: utterance draw, crop offset only for long utterances, zero padding);
  * one get_loader epoch (data_loader.py:88-102): torch.manual_seed(99), np.random.seed(4321),
    batch_size 2, shuffle, drop_last, num_workers 0.

  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_data_goldens.py
"""
import os
import pickle
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LEN_CROP = 32
ORDER = [3, 0, 4, 1, 1, 2, 0, 3, 4, 2] * 5


def build_tree(root, len_crop=LEN_CROP):
    """The miniature VCTK-layout dataset (train.pkl + spk/utt.npy), deterministic."""
    rng = np.random.RandomState(7)
    meta = []
    for s in range(5):
        spk = f"p{225 + s}"
        os.makedirs(os.path.join(root, spk), exist_ok=True)
        emb = rng.randn(256).astype(np.float32)
        entry = [spk, emb]
        for u in range(2 + s % 3):
            T = [len_crop - 9, len_crop, len_crop + 1, 3 * len_crop + 5][(s + u) % 4]
            mel = (rng.rand(T, 80) * 7 - 5).astype(np.float32)
            rel = f"{spk}/{spk}_{u:03d}.npy"
            np.save(os.path.join(root, rel), mel)
            entry.append(rel.replace("/", "\\") if (s, u) == (1, 0) else rel)
        meta.append(entry)
    with open(os.path.join(root, "train.pkl"), "wb") as f:
        pickle.dump(meta, f)
    return meta


def main():
    import torch

    sys.path.insert(0, "/root/reference")
    from util.data_loader import Utterances, get_loader  # the reference itself

    rec = {}
    with tempfile.TemporaryDirectory() as root:
        build_tree(root)
        ds = Utterances(root, LEN_CROP)
        np.random.seed(1234)
        items = [ds[i] for i in ORDER]
        rec["item_uttr"] = np.stack([u for u, _ in items]).astype(np.float32)
        rec["item_emb"] = np.stack([e for _, e in items]).astype(np.float32)
        rec["order"] = np.array(ORDER)
        torch.manual_seed(99)
        np.random.seed(4321)
        loader = get_loader(root, batch_size=2, len_crop=LEN_CROP)
        xs, es = [], []
        for x, e in loader:
            xs.append(x.numpy())
            es.append(e.numpy())
        rec["epoch_x"] = np.stack(xs).astype(np.float32)
        rec["epoch_emb"] = np.stack(es).astype(np.float32)
    out = os.path.join(HERE, "data_ref.npz")
    np.savez_compressed(out, **rec)
    print("wrote", out, {k: v.shape for k, v in rec.items()})


if __name__ == "__main__":
    main()
