"""Pin the CPU oracle against goldens generated from the reference."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import autovc_cpu as A
from oracle import discriminator_cpu as D
from oracle import metaformer_cpu as M

from .conftest import GOLDEN

torch.set_num_threads(min(8, os.cpu_count() or 1))


def rel_inf(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)


def _layout():
    with open(os.path.join(GOLDEN, "state_dict_layout.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name,spec", [("AutoVC", A.autovc_spec), ("MetaConv", M.metaconv_spec),
                                       ("MetaPool", M.metapool_spec), ("Discriminator", D.disc_spec)])
def test_spec_matches_reference_layout(name, spec):
    ref = [(k, tuple(s)) for k, s in _layout()[name]]
    ours = [(k, tuple(s)) for k, s in spec().items()]
    assert ours == ref


def _run_step(fname, spec_fn, fwd):
    g = np.load(os.path.join(GOLDEN, fname))
    freq = int(g["freq"])
    sd = A.make_state(spec_fn())
    x, e = torch.from_numpy(g["x"]), torch.from_numpy(g["emb"])
    losses, total, outs = A.step_losses(lambda a, b, c: fwd(sd, a, b, c, dim_neck=44, freq=freq), x, e)
    total.backward()
    return g, sd, losses, outs


@pytest.mark.parametrize("fname", ["autovc_T176.npz", "autovc_T128.npz"])
def test_autovc_oracle_forward_backward(fname):
    g, sd, losses, outs = _run_step(fname, A.autovc_spec, A.autovc_forward)
    assert rel_inf(outs[0].detach().numpy(), g["mel"]) < 1e-5
    assert rel_inf(outs[1].detach().numpy(), g["mel_psnt"]) < 1e-5
    assert rel_inf(outs[2].detach().numpy(), g["codes"]) < 1e-5
    assert rel_inf(outs[3].detach().numpy(), g["codes_re"]) < 1e-5
    np.testing.assert_allclose([l.item() for l in losses], g["losses"], rtol=1e-5)
    for k, t in sd.items():
        if t.requires_grad:
            gn = float(g["gnorm/" + k])
            ours = t.grad.norm().item()
            assert abs(ours - gn) <= 1e-3 * gn + 1e-6, (k, ours, gn)
            head = t.grad.reshape(-1)[:64].numpy()
            assert np.abs(head - g["ghead/" + k]).max() <= 1e-3 * max(np.abs(g["ghead/" + k]).max(), 1e-3), k
        elif "running" in k or "num_batches" in k:
            np.testing.assert_allclose(t.numpy(), g["bn/" + k], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("fname,freq", [("autovc_T176.npz", 22), ("autovc_T128.npz", 16)])
def test_oracle_solver_three_adam_steps(fname, freq):
    g = np.load(os.path.join(GOLDEN, fname))
    s = A.OracleSolver(freq=freq)
    got = [s.step(torch.from_numpy(g[f"adam_x{i}"]), torch.from_numpy(g[f"adam_e{i}"])) for i in range(3)]
    np.testing.assert_allclose(np.array(got), g["adam_losses"], rtol=1e-4)
    for k, t in s.sd.items():
        if t.requires_grad:
            np.testing.assert_allclose(t.detach().reshape(-1)[:64].numpy(), g["after/" + k], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("fname,spec,fwd", [("metaconv_T176.npz", M.metaconv_spec, M.metaconv_forward),
                                            ("metapool_T176.npz", M.metapool_spec, M.metapool_forward)])
def test_metaformer_oracle(fname, spec, fwd):
    g, sd, losses, outs = _run_step(fname, spec, fwd)
    assert rel_inf(outs[1].detach().numpy(), g["mel_psnt"]) < 1e-5
    assert rel_inf(outs[2].detach().numpy(), g["codes"]) < 1e-5
    assert rel_inf(outs[3].detach().numpy(), g["codes_re"]) < 1e-5
    np.testing.assert_allclose([l.item() for l in losses], g["losses"], rtol=1e-5)
    for k, t in sd.items():
        if t.requires_grad:
            gn = float(g["gnorm/" + k])
            assert abs(t.grad.norm().item() - gn) <= 2e-3 * gn + 1e-6, k


def test_discriminator_oracle():
    g = np.load(os.path.join(GOLDEN, "disc_T176.npz"))
    sd = A.make_state(A.autovc_spec())
    dsd = A.make_state(D.disc_spec())
    x, e = torch.from_numpy(g["x"]), torch.from_numpy(g["emb"])
    losses, total, outs = A.step_losses(lambda a, b, c: A.autovc_forward(sd, a, b, c, freq=22), x, e)
    real = D.disc_forward(dsd, x)
    fake = D.disc_forward(dsd, outs[1].squeeze())
    dl = D.discriminator_loss(real, fake)
    (total + dl).backward()
    np.testing.assert_allclose(real.detach().numpy(), g["real"], rtol=1e-5)
    np.testing.assert_allclose(fake.detach().numpy(), g["fake"], rtol=1e-5)
    np.testing.assert_allclose(dl.item(), g["d_loss"], rtol=1e-5)
    for k, t in dsd.items():
        if t.requires_grad:
            gn = float(g["dgnorm/" + k])
            assert abs(t.grad.norm().item() - gn) <= 1e-3 * gn + 1e-6, k


def test_gan_solver_three_steps():
    g = np.load(os.path.join(GOLDEN, "disc_T176.npz"))
    s = D.OracleGANSolver(freq=22)
    got = [s.step(torch.from_numpy(g[f"adam_x{i}"]), torch.from_numpy(g[f"adam_e{i}"]))[3] for i in range(3)]
    np.testing.assert_allclose(got, g["d_step_losses"], rtol=1e-4)


def test_lstm_loop_matches_torch_lstm():
    torch.manual_seed(0)
    B, T, I, H = 3, 7, 5, 4
    x = torch.randn(B, T, I)
    w = [torch.randn(4 * H, I), torch.randn(4 * H, H), torch.randn(4 * H), torch.randn(4 * H)]
    sd = {"l.weight_ih_l0": w[0], "l.weight_hh_l0": w[1], "l.bias_ih_l0": w[2], "l.bias_hh_l0": w[3]}
    ref = A.lstm(x, sd, "l", H, 1, False)
    np.testing.assert_allclose(A.lstm_loop(x, *w).numpy(), ref.numpy(), rtol=1e-5, atol=1e-6)
