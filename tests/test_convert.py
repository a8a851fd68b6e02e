"""Conversion path (autoformer_amd/convert.py, reference util/evaluate.py:36-94): crop/pad
bookkeeping on the host, and (GPU) one-utterance conversion with a target speaker different
from the source against the CPU oracle's AutoVC forward (fp32 compute mode)."""
import numpy as np
import pytest
import torch


def test_crop_mel_bookkeeping():
    from autoformer_amd.convert import crop_mel

    rng = np.random.RandomState(3)
    short = rng.rand(50, 80).astype(np.float32)
    out, pad = crop_mel(short, 64)
    assert out.shape == (64, 80) and pad == 14
    np.testing.assert_array_equal(out[:50], short)
    assert not out[50:].any()
    exact = rng.rand(64, 80).astype(np.float32)
    out, pad = crop_mel(exact, 64)
    assert pad == 0 and out is exact
    long = rng.rand(100, 80).astype(np.float32)
    np.random.seed(5)
    out, pad = crop_mel(long, 64)
    np.random.seed(5)
    left = np.random.randint(0, 100 - 64)
    assert pad == 0
    np.testing.assert_array_equal(out, long[left:left + 64])


@pytest.mark.gpu
def test_convert_matches_oracle_with_other_target_speaker():
    import autoformer_amd as A
    from autoformer_amd.convert import Converter
    from autoformer_amd.detinit import det_init_, det_inputs
    from autoformer_amd.factory.AutoVC import AutoVC
    from oracle import autovc_cpu as O

    T, freq = 64, 16
    x, e = det_inputs(2, T, seed=21)
    src, emb_org, emb_trg = x[0][: T - 10], e[0], e[1]  # source shorter than len_crop: padded
    A.set_compute("fp32")
    m = AutoVC(44, 256, 512, freq)
    det_init_(m)
    m = m.cuda().train()
    got = Converter(m, T).convert(src, emb_org, emb_trg)
    assert got.shape == (T - 10, 80)
    sd = O.make_state(O.autovc_spec())
    xp = np.zeros((1, T, 80), np.float32)
    xp[0, : T - 10] = src
    with torch.no_grad():
        outs = O.autovc_forward(sd, torch.from_numpy(xp), torch.from_numpy(emb_org[None]),
                                torch.from_numpy(emb_trg[None]), freq=freq)
    ref = outs[1].squeeze(1)[0, : T - 10].numpy()
    rel = np.abs(got - ref).max() / np.abs(ref).max()
    assert rel < 1e-3, rel
