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


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["AutoVC_Adjust", "AutoVC2", "MetaConv2"])
def test_converter_dispatch_matches_reference_get_trans_mel(name):
    """Converter.get_trans_mel dispatches like util/evaluate.py:77-83: isAdjust ->
    model(x, e_org, e_trg, True, mel_target); isAdain -> model(x, e_org, None, None) for the
    source features, then model(x, e_org, e_trg, feature).  Same result as those calls made by
    hand on an identically initialised model (train-mode BN, as the reference converts)."""
    from autoformer_amd.convert import Converter
    from tests.test_variants import _golden, _variant_model

    dev = torch.device("cuda:0")
    g = _golden(name)
    x, e, x2, e2 = (g[k] for k in ("x", "emb", "x2", "emb2"))
    T = x.shape[1]
    adjust = name.endswith("_Adjust")
    m1, m2 = _variant_model(name, dev), _variant_model(name, dev)
    src, mt, trans = Converter(m1, T, dev).get_trans_mel(x[0], x2[0], e[0], e2[0], isAdjust=adjust,
                                                         isAdain=not adjust)
    xs, xt = torch.from_numpy(x[:1]).to(dev), torch.from_numpy(x2[:1]).to(dev)
    eo, et = torch.from_numpy(e[:1]).to(dev), torch.from_numpy(e2[:1]).to(dev)
    with torch.no_grad():
        if adjust:
            _, _, ref, _ = m2(xs, eo, et, True, xt)
        else:
            _, feature = m2(xs, eo, None, None)
            _, ref, _ = m2(xs, eo, et, feature)
    torch.testing.assert_close(src, xs)
    torch.testing.assert_close(mt, xt)
    torch.testing.assert_close(trans, ref.squeeze(1), rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_converter_get_wavs_end_to_end():
    """evaluate.py:56-98 in one chain on the device: convert (AutoVC, padded source, other target
    speaker), trim, vocode the frame-major converted mel with the HIP MelGAN generator; the
    waveform equals the oracle generator on the same converted mel (fp32 compute mode), and the
    (1, 80, T) entry of get_wavs gives the same samples."""
    import autoformer_amd as A
    from autoformer_amd.convert import Converter
    from autoformer_amd.detinit import det_init_, det_inputs, det_melgan_state
    from autoformer_amd.factory.AutoVC import AutoVC
    from autoformer_amd.melgan import Generator, MelVocoder
    from oracle import melgan_cpu as OM

    T, freq = 64, 16
    x, e = det_inputs(2, T, seed=23)
    A.set_compute("fp32")
    try:
        m = AutoVC(44, 256, 512, freq)
        det_init_(m)
        g = Generator(80, 32, 3)
        sd = {k: torch.from_numpy(v) for k, v in
              det_melgan_state([(k, tuple(v.shape)) for k, v in g.state_dict().items()]).items()}
        g.load_state_dict(sd)
        conv = Converter(m.cuda().train(), T, vocoder=MelVocoder(generator=g))
        _, _, mel = conv.get_trans_mel(x[0][: T - 6], None, e[0], e[1], isPlay=True)  # (1, T-6, 80)
        wav = conv.get_wavs(mel, frames=True)
        wav2 = conv.get_wavs(mel.transpose(1, 2).contiguous())
        torch.cuda.synchronize()
        assert wav.shape == (1, (T - 6) * 256)
        ref = OM.generator(sd, mel.transpose(1, 2).cpu()).squeeze(1)
        assert (wav.cpu() - ref).abs().max() / ref.abs().max() < 1e-4
        assert torch.equal(wav, wav2)
    finally:
        A.set_compute("bf16")


def test_get_wavs_layout_is_stated_not_guessed():
    """a frame-major mel with T == 80 is vocoded frame-major only when the caller says
    so (frames=True); the default is the reference's (1, 80, T) contract; a wrong layout raises."""
    from autoformer_amd.convert import Converter

    class Voc:
        def inverse(self, m):
            return ("inverse", tuple(m.shape))

        def inverse_frames(self, m):
            return ("frames", tuple(m.shape))

    c = Converter(None, 80, device="cpu", vocoder=Voc())
    sq = torch.zeros(1, 80, 80)
    assert c.get_wavs(sq) == ("inverse", (1, 80, 80))
    assert c.get_wavs(sq, frames=True) == ("frames", (1, 80, 80))
    assert c.get_wavs(torch.zeros(1, 80, 64)) == ("inverse", (1, 80, 64))
    assert c.get_wavs(torch.zeros(1, 64, 80), frames=True) == ("frames", (1, 64, 80))
    with pytest.raises(ValueError):
        c.get_wavs(torch.zeros(1, 64, 80))
    with pytest.raises(ValueError):
        c.get_wavs(torch.zeros(1, 80, 64), frames=True)
