"""MelGAN vocoder generator (reference melgan/modules.py:88-131).

CPU: the oracle restatement (oracle/melgan_cpu.py) against the fixture generated from the
reference module itself (tests/golden/make_melgan_goldens.py); the build's state_dict layout;
the polyphase ConvTranspose1d decomposition the HIP pack uses (index maths restated in torch)
against F.conv_transpose1d.
GPU: the HIP Generator (fp32 and bf16 compute) against the fixture and the oracle.
Bars: fp32 rel-inf <= 1e-4 (fp32 MFMA, fp32 accumulation; oracle vs reference 1.3e-6);
bf16 rel-inf <= 5e-2 (the build's bf16 bar)."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import melgan_cpu as O

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "melgan_G.npz"))


def _sd():
    from autoformer_amd.detinit import det_melgan_state

    shapes = [(k, tuple(int(v) for v in s.split(","))) for k, s in zip(G["keys"], G["shapes"])]
    return {k: torch.from_numpy(v) for k, v in det_melgan_state(shapes).items()}


def _rel_inf(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.abs(a - b).max() / np.abs(b).max()


def test_oracle_matches_reference_fixture():
    out = O.generator(_sd(), torch.from_numpy(G["mel"]))
    assert out.shape == G["audio"].shape
    assert _rel_inf(out.numpy(), G["audio"]) < 1e-5


def test_state_dict_layout_matches_reference():
    from autoformer_amd.melgan import Generator

    sd = Generator(80, 32, 3).state_dict()
    assert list(sd.keys()) == list(G["keys"])
    assert [",".join(map(str, v.shape)) for v in sd.values()] == list(G["shapes"])


@pytest.mark.parametrize("r", [8, 2])
def test_polyphase_conv_transpose_decomposition(r):
    """ConvTranspose1d(k = 2r, stride r, padding r/2 + r%2) == ONE product over the zero-padded
    3-tap window (j-1, j, j+1) with phase-major columns (p, co): the pack of avc_mg_wn_pack."""
    torch.manual_seed(r)
    Ci, Co, L, pad = 6, 5, 9, r // 2 + r % 2
    x = torch.randn(2, Ci, L, dtype=torch.float64)
    w = torch.randn(Ci, Co, 2 * r, dtype=torch.float64)
    ref = F.conv_transpose1d(x, w, stride=r, padding=pad, output_padding=r % 2)
    Wp = torch.zeros(r * Co, 3 * Ci, dtype=torch.float64)
    for p in range(r):
        dl, rho = (p + pad) // r, (p + pad) % r
        for co in range(Co):
            Wp[p * Co + co, (dl + 1) * Ci:(dl + 2) * Ci] = w[:, co, rho]
            Wp[p * Co + co, dl * Ci:(dl + 1) * Ci] = w[:, co, rho + r]
    xf = F.pad(x, (1, 1)).transpose(1, 2)                   # (B, L+2, Ci), zero-padded
    A = torch.cat([xf[:, t:t + L] for t in range(3)], -1)   # (B, L, 3Ci): taps j-1, j, j+1
    out = (A @ Wp.T).reshape(2, L * r, Co).transpose(1, 2)  # [B*L][r*Co] == [B*L*r][Co]
    assert out.shape == ref.shape
    assert (out - ref).abs().max() < 1e-12


# ------------------------------------------------------------------------------------- GPU
def _gen(comp):
    import autoformer_amd as A
    from autoformer_amd.melgan import Generator

    A.set_compute(comp)
    g = Generator(80, 32, 3)
    g.load_state_dict(_sd())
    return g.to("cuda:0")


@pytest.mark.gpu
@pytest.mark.parametrize("comp,tol", [("fp32", 1e-4), ("bf16", 5e-2)])
def test_hip_generator_matches_reference_fixture(comp, tol):
    g = _gen(comp)
    try:
        out = g(torch.from_numpy(G["mel"]).cuda())
        torch.cuda.synchronize()
        assert out.shape == G["audio"].shape
        assert _rel_inf(out.cpu().numpy(), G["audio"]) < tol
    finally:
        import autoformer_amd as A

        A.set_compute("bf16")


@pytest.mark.gpu
def test_hip_generator_matches_oracle_other_shapes():
    """B = 3, T = 37 (odd, not a multiple of anything) in fp32; and the frame-major entry
    (MelVocoder.inverse_frames, the Converter's (B, T, 80) layout) equals inverse()."""
    from autoformer_amd.detinit import det_mel
    from autoformer_amd.melgan import MelVocoder

    g = _gen("fp32")
    try:
        mel = torch.from_numpy(det_mel(3, 80, 37, seed=7))
        ref = O.generator(_sd(), mel)
        voc = MelVocoder(generator=g)
        out = voc.inverse(mel.cuda())
        outf = voc.inverse_frames(mel.transpose(1, 2).contiguous().cuda())
        torch.cuda.synchronize()
        assert out.shape == (3, 37 * 256)
        assert _rel_inf(out.cpu().numpy(), ref.squeeze(1).numpy()) < 1e-4
        assert torch.equal(out, outf)
    finally:
        import autoformer_amd as A

        A.set_compute("bf16")


@pytest.mark.gpu
def test_hip_generator_refuses_short_input():
    g = _gen("bf16")
    with pytest.raises(ValueError):
        g.frames(torch.zeros(3, 80, device="cuda:0"), 1, 3)
