"""Discriminator + two-model step parity on the MI355X against disc_T176.npz (generated
from /root/reference/factory/Discriminator.py and train_with_discriminator.Solver)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _models(comp="fp32"):
    import autoformer_amd as A
    from autoformer_amd.detinit import det_init_
    from factory.AutoVC import AutoVC
    from factory.Discriminator import Discriminator

    A.set_compute(comp)
    G, Dm = AutoVC(44, 256, 512, 22), Discriminator()
    det_init_(G)
    det_init_(Dm)
    return G.to(DEV).train(), Dm.to(DEV).train()


def test_discriminator_forward_backward_matches_reference(golden):
    from autoformer_amd.train import discriminator_loss, vc_losses

    g = golden("disc_T176.npz")
    G, Dm = _models()
    x, e = torch.from_numpy(g["x"]).to(DEV), torch.from_numpy(g["emb"]).to(DEV)
    loss, parts, x_psnt = vc_losses(G, x, e)
    real = Dm(x)
    fake = Dm(x_psnt.squeeze())
    dl = discriminator_loss(real, fake)
    (loss + dl).backward()
    torch.cuda.synchronize()
    np.testing.assert_allclose(real.detach().cpu().numpy(), g["real"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(fake.detach().cpu().numpy(), g["fake"], rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(dl.item(), float(g["d_loss"]), rtol=1e-4)
    np.testing.assert_allclose([p.item() for p in parts], g["g_losses"], rtol=1e-4)
    for name, p in Dm.named_parameters():
        ref = float(g["dgnorm/" + name])
        assert abs(p.grad.norm().item() - ref) <= 1e-2 * ref + 1e-6, (name, p.grad.norm().item(), ref)
    for k, v in Dm.state_dict().items():
        if "running" in k or "num_batches" in k:
            assert v.shape == g["dsd/" + k].shape


def test_gan_three_steps_match_reference_solver(golden):
    """train_with_discriminator.Solver: one loss for G and D, both Adams step (torch Adam here)."""
    from autoformer_amd.train import discriminator_loss, vc_losses

    g = golden("disc_T176.npz")
    G, Dm = _models()
    og = torch.optim.Adam(G.parameters(), 1e-4)
    od = torch.optim.Adam(Dm.parameters(), 1e-4)
    got = []
    for i in range(3):
        x = torch.from_numpy(g[f"adam_x{i}"]).to(DEV)
        e = torch.from_numpy(g[f"adam_e{i}"]).to(DEV)
        loss, parts, x_psnt = vc_losses(G, x, e)
        dl = discriminator_loss(Dm(x), Dm(x_psnt.squeeze()))
        og.zero_grad()
        od.zero_grad()
        (loss + dl).backward()
        og.step()
        od.step()
        got.append(dl.item())
    np.testing.assert_allclose(got, g["d_step_losses"], rtol=2e-3)


def test_gan_trainstep_bf16_runs():
    from autoformer_amd.detinit import det_inputs
    from autoformer_amd.layers import set_grad_sink
    from autoformer_amd.train import TrainStep, gan_extra

    G, Dm = _models("bf16")
    x, e = det_inputs(8, 176, seed=5)
    x, e = torch.from_numpy(x).to(DEV), torch.from_numpy(e).to(DEV)
    ts = TrainStep(G, extra=gan_extra(Dm), extra_modules=[Dm])
    try:
        losses = [ts.step(x, e).item() for _ in range(3)]
    finally:
        set_grad_sink(False)
    assert all(np.isfinite(losses)) and losses[-1] < losses[0]
