"""The training-data path (autoformer_amd/data.py, reference util/data_loader.py): on-disk
format, sampling parity with the restated reference (oracle/data_cpu.py) under one numpy seed,
the DataLoader contract, and (GPU) the pinned / copy-stream device feed."""
import os
import pickle

import numpy as np
import pytest
import torch

from oracle.data_cpu import reference_item

LEN_CROP = 32


@pytest.fixture(scope="module")
def vctk_like(tmp_path_factory):
    """A miniature dataset in the reference layout: 5 speakers, 2-4 utterances each, lengths
    shorter than, equal to and longer than len_crop; one path written with a backslash."""
    root = tmp_path_factory.mktemp("vctk")
    rng = np.random.RandomState(7)
    meta, mels = [], {}
    for s in range(5):
        spk = f"p{225 + s}"
        os.makedirs(root / spk)
        emb = rng.randn(256).astype(np.float32)
        entry = [spk, emb]
        for u in range(2 + s % 3):
            T = [LEN_CROP - 9, LEN_CROP, LEN_CROP + 1, 3 * LEN_CROP + 5][(s + u) % 4]
            mel = (rng.rand(T, 80) * 7 - 5).astype(np.float32)
            rel = f"{spk}/{spk}_{u:03d}.npy"
            np.save(root / rel, mel)
            mels[rel] = mel
            entry.append(rel.replace("/", "\\") if (s, u) == (1, 0) else rel)
        meta.append(entry)
    with open(root / "train.pkl", "wb") as f:
        pickle.dump(meta, f)
    return str(root), meta, mels


def test_utterances_load_reference_layout(vctk_like):
    from autoformer_amd.data import Utterances

    root, meta, mels = vctk_like
    ds = Utterances(root, LEN_CROP)
    assert len(ds) == len(meta)
    for entry, got in zip(meta, ds.train_dataset):
        assert got[0] == entry[0]
        np.testing.assert_array_equal(got[1], entry[1])
        for rel, mel in zip(entry[2:], got[2:]):
            np.testing.assert_array_equal(mel, mels[rel.replace("\\", "/")])


def test_item_sampling_matches_reference_under_one_seed(vctk_like):
    from autoformer_amd.data import Utterances

    root, meta, _ = vctk_like
    ds = Utterances(root, LEN_CROP)
    order = [3, 0, 4, 1, 1, 2, 0, 3, 4, 2] * 5
    np.random.seed(1234)
    got = [ds[i] for i in order]
    np.random.seed(1234)
    ref = [reference_item(ds.train_dataset[i], LEN_CROP) for i in order]
    for (gu, ge), (ru, re) in zip(got, ref):
        assert gu.shape == (LEN_CROP, 80) and gu.dtype == np.float32
        np.testing.assert_array_equal(gu, ru)
        np.testing.assert_array_equal(ge, re)


def test_get_loader_contract(vctk_like):
    from autoformer_amd.data import get_loader

    root, meta, _ = vctk_like
    loader = get_loader(root, batch_size=2, len_crop=LEN_CROP)
    batches = list(loader)
    assert len(batches) == len(meta) // 2  # drop_last
    for uttr, emb in batches:
        assert uttr.shape == (2, LEN_CROP, 80) and uttr.dtype == torch.float32
        assert emb.shape == (2, 256) and emb.dtype == torch.float32


@pytest.mark.gpu
def test_device_feed_matches_host_batches(vctk_like):
    from autoformer_amd.data import DeviceFeed, get_loader

    root, _, _ = vctk_like
    torch.manual_seed(0)
    np.random.seed(0)
    host = [(u.clone(), e.clone()) for u, e in get_loader(root, batch_size=2, len_crop=LEN_CROP)]
    torch.manual_seed(0)
    np.random.seed(0)
    feed = DeviceFeed(get_loader(root, batch_size=2, len_crop=LEN_CROP), "cuda:0")
    dev = [(x.cpu(), e.cpu()) for x, e in feed]
    assert len(dev) == len(host)
    for (hx, he), (dx, de) in zip(host, dev):
        torch.testing.assert_close(dx, hx, rtol=0, atol=0)
        torch.testing.assert_close(de, he, rtol=0, atol=0)


# ---------------------------------------------------------------- pinned to the reference itself
# tests/golden/data_ref.npz was written by the reference's own util/data_loader.py
# (tests/golden/make_data_goldens.py) over the tree build_tree() makes.
def _ref_tree(tmp_path):
    from tests.golden.make_data_goldens import build_tree

    root = str(tmp_path)
    build_tree(root)
    return root


def test_items_match_reference_loader_fixture(tmp_path, golden):
    from autoformer_amd.data import Utterances
    from tests.golden.make_data_goldens import LEN_CROP as LC

    g = golden("data_ref.npz")
    ds = Utterances(_ref_tree(tmp_path), LC)
    np.random.seed(1234)
    got = [ds[int(i)] for i in g["order"]]
    np.testing.assert_array_equal(np.stack([u for u, _ in got]), g["item_uttr"])
    np.testing.assert_array_equal(np.stack([e for _, e in got]), g["item_emb"])


def test_loader_epoch_matches_reference_loader_fixture(tmp_path, golden):
    from autoformer_amd.data import get_loader
    from tests.golden.make_data_goldens import LEN_CROP as LC

    g = golden("data_ref.npz")
    root = _ref_tree(tmp_path)
    torch.manual_seed(99)
    np.random.seed(4321)
    batches = list(get_loader(root, batch_size=2, len_crop=LC))
    np.testing.assert_array_equal(np.stack([x.numpy() for x, _ in batches]), g["epoch_x"])
    np.testing.assert_array_equal(np.stack([e.numpy() for _, e in batches]), g["epoch_emb"])
