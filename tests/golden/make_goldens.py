"""Generate golden fixtures from the *reference* modules (survey container only).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_goldens.py

This script imports achyun/Autoformer from /root/reference (read-only) on the
CPU, loads the closed-form deterministic weights of autoformer_amd.detinit into
it, runs the hot path and writes small .npz fixtures next to this file.  The
reference never travels to the GPU box; only these arrays do.

Fixtures:
  autovc_T176.npz   G1/G3/G4  AutoVC B=2 T=176 freq=22 (train.py defaults)
  autovc_T128.npz   G2/G3/G4  AutoVC B=2 T=128 freq=16 (metric shape family)
  metaconv_T176.npz G5        MetaConv B=2 T=176
  metapool_T176.npz G5        MetaPool B=2 T=176
  disc_T176.npz     G6        Discriminator on G1's tensors + 3-step two-model losses
"""
import os
import sys
import types

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
REF = "/root/reference"

sys.dont_write_bytecode = True
sys.path.insert(0, REPO)
from autoformer_amd.detinit import det_init_, det_inputs  # noqa: E402

sys.path.insert(0, REF)
sys.modules.setdefault("wandb", types.SimpleNamespace(log=lambda *a, **k: None,
                                                      save=lambda *a, **k: None,
                                                      init=lambda *a, **k: None))
torch.manual_seed(0)
torch.set_num_threads(8)


def _grads(model):
    out = {}
    for name, p in model.named_parameters():
        g = p.grad if p.grad is not None else torch.zeros_like(p)
        out["gnorm/" + name] = np.array(g.norm().item(), dtype=np.float64)
        out["ghead/" + name] = g.detach().reshape(-1)[:64].numpy().copy()
    return out


def _bn_stats(model):
    out = {}
    for k, v in model.state_dict().items():
        if "running_" in k or "num_batches_tracked" in k:
            out["bn/" + k] = v.detach().numpy().copy()
    return out


def _g_step(model, x, e):
    """One step of train.py:Solver.train (/root/reference/train.py:82-99), no optimizer."""
    model.train()
    x_id, x_id_psnt, code_real = model(x, e, e)
    l_id = F.mse_loss(x, x_id.squeeze())
    l_id_psnt = F.mse_loss(x, x_id_psnt.squeeze())
    code_re = model(x_id_psnt, e, None)
    l_cd = F.l1_loss(code_real, code_re)
    loss = l_id + l_id_psnt + 1.0 * l_cd
    return (x_id, x_id_psnt, code_real, code_re), (l_id, l_id_psnt, l_cd), loss


def make_autovc_like(modname, clsname, T, freq, fname, steps=3):
    mod = __import__(f"factory.{modname}", fromlist=[clsname])
    model = getattr(mod, clsname)(44, 256, 512, freq)
    det_init_(model)
    x, e = det_inputs(2, T)
    xt, et = torch.from_numpy(x), torch.from_numpy(e)
    outs, losses, loss = _g_step(model, xt, et)
    model.zero_grad()
    loss.backward()
    rec = {
        "x": x, "emb": e, "T": np.array(T), "freq": np.array(freq),
        "mel": outs[0].detach().numpy(), "mel_psnt": outs[1].detach().numpy(),
        "codes": outs[2].detach().numpy(), "codes_re": outs[3].detach().numpy(),
        "losses": np.array([l.item() for l in losses], dtype=np.float64),
    }
    rec.update(_grads(model))
    rec.update(_bn_stats(model))

    # G4: losses of `steps` Adam steps through the reference Solver itself.
    if steps:
        import importlib
        train = importlib.import_module("train")
        cfg = train.Config(model_name=modname, data_dir=None, device="cpu",
                           num_iters=steps, isadain=False)
        cfg.freq = freq
        cfg.batch_size = 2
        cfg.len_crop = T
        batches = [(torch.from_numpy(det_inputs(2, T, seed=100 + i)[0]),
                    torch.from_numpy(det_inputs(2, T, seed=100 + i)[1])) for i in range(steps)]
        solver = train.Solver(batches, cfg)
        det_init_(solver.VC)
        seen = []
        orig = F.l1_loss

        def spy(a, b, *args, **kw):
            r = orig(a, b, *args, **kw)
            seen.append(r.item())
            return r
        F.l1_loss = spy
        try:
            # record every loss with a light hook on mse/l1 via re-running the step formula
            solver_losses = []
            orig_mse = F.mse_loss

            def spy_mse(a, b, *args, **kw):
                r = orig_mse(a, b, *args, **kw)
                solver_losses.append(r.item())
                return r
            F.mse_loss = spy_mse
            train.F.mse_loss = spy_mse
            train.F.l1_loss = spy
            solver.train()
        finally:
            F.l1_loss = orig
            F.mse_loss = orig_mse
            train.F.mse_loss = orig_mse
            train.F.l1_loss = orig
        steps_losses = np.array(
            [[solver_losses[2 * i], solver_losses[2 * i + 1], seen[i]] for i in range(steps)])
        rec["adam_losses"] = steps_losses
        for i in range(steps):
            rec[f"adam_x{i}"] = batches[i][0].numpy()
            rec[f"adam_e{i}"] = batches[i][1].numpy()
        # a few parameter tensors after the 3 steps (heads)
        for name, p in solver.VC.named_parameters():
            rec["after/" + name] = p.detach().reshape(-1)[:64].numpy().copy()
    np.savez_compressed(os.path.join(HERE, fname), **rec)
    print("wrote", fname, {k: v.shape for k, v in rec.items() if not k.startswith(("g", "bn/", "after/"))})
    return model, outs


def make_disc(fname, steps=3):
    from factory.Discriminator import Discriminator
    import factory.AutoVC as A
    G = A.AutoVC(44, 256, 512, 22)
    D = Discriminator()
    det_init_(G)
    det_init_(D)
    x, e = det_inputs(2, 176, seed=77)
    xt, et = torch.from_numpy(x), torch.from_numpy(e)
    outs, losses, loss = _g_step(G, xt, et)
    real = D(xt)
    fake = D(outs[1].squeeze())
    bce = torch.nn.BCELoss()
    d_loss = bce(real, torch.ones_like(real)) + bce(fake, torch.zeros_like(fake))
    total = loss + d_loss
    G.zero_grad(); D.zero_grad()
    total.backward()
    rec = {"x": x, "emb": e, "real": real.detach().numpy(), "fake": fake.detach().numpy(),
           "d_loss": np.array(d_loss.item()), "g_losses": np.array([l.item() for l in losses])}
    for name, p in D.named_parameters():
        rec["dgnorm/" + name] = np.array(p.grad.norm().item())
        rec["dghead/" + name] = p.grad.reshape(-1)[:64].numpy().copy()
    for k, v in D.state_dict().items():
        rec["dsd/" + k] = v.numpy().copy()
    # 3 steps of train_with_discriminator.Solver (shared loss, two Adams)
    import importlib
    twd = importlib.import_module("train_with_discriminator")
    cfg = twd.Config("AutoVC", None, steps)
    batches = [(torch.from_numpy(det_inputs(2, 176, seed=200 + i)[0]),
                torch.from_numpy(det_inputs(2, 176, seed=200 + i)[1])) for i in range(steps)]
    solver = twd.Solver(batches, cfg)
    det_init_(solver.G)
    det_init_(solver.D)
    seen = []
    orig_bce_fwd = torch.nn.BCELoss.forward

    def spy(self, a, b):
        r = orig_bce_fwd(self, a, b)
        seen.append(r.item())
        return r
    torch.nn.BCELoss.forward = spy
    try:
        solver.train()
    finally:
        torch.nn.BCELoss.forward = orig_bce_fwd
    rec["d_step_losses"] = np.array([seen[2 * i] + seen[2 * i + 1] for i in range(steps)])
    for i in range(steps):
        rec[f"adam_x{i}"] = batches[i][0].numpy()
        rec[f"adam_e{i}"] = batches[i][1].numpy()
    for name, p in solver.D.named_parameters():
        rec["dafter/" + name] = p.detach().reshape(-1)[:64].numpy().copy()
    np.savez_compressed(os.path.join(HERE, fname), **rec)
    print("wrote", fname)


def main():
    make_autovc_like("AutoVC", "AutoVC", 176, 22, "autovc_T176.npz")
    make_autovc_like("AutoVC", "AutoVC", 128, 16, "autovc_T128.npz")
    make_autovc_like("MetaConv", "MetaConv", 176, 22, "metaconv_T176.npz", steps=0)
    make_autovc_like("MetaPool", "MetaPool", 176, 22, "metapool_T176.npz", steps=0)
    make_disc("disc_T176.npz")


def dump_state_dict_layout(fname="state_dict_layout.json"):
    """Reference state_dict keys + shapes (the drop-in contract)."""
    import json
    import factory.AutoVC as A
    import factory.MetaConv as MC
    import factory.MetaPool as MP
    from factory.Discriminator import Discriminator
    out = {}
    for name, m in [("AutoVC", A.AutoVC(44, 256, 512, 22)), ("MetaConv", MC.MetaConv(44, 256, 512, 22)),
                    ("MetaPool", MP.MetaPool(44, 256, 512, 22)), ("Discriminator", Discriminator())]:
        out[name] = [[k, list(v.shape)] for k, v in m.state_dict().items()]
    with open(os.path.join(HERE, fname), "w") as f:
        json.dump(out, f)
    print("wrote", fname, {k: len(v) for k, v in out.items()})


if __name__ == "__main__":
    if "--layout-only" not in sys.argv:
        main()
    dump_state_dict_layout()
