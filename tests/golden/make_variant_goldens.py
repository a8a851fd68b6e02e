"""Generate golden fixtures for the AdaIN / Adjust model variants from the *reference*
modules (survey container only).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_variant_goldens.py

Imports achyun/Autoformer's factory.{AutoVC2, MetaConv2, MetaPool2, AutoVC_Adjust,
MetaConv_Adjust, MetaPool_Adjust} from /root/reference (read-only) on the CPU, loads the
closed-form weights of autoformer_amd.detinit and records, per model, B=2, T=176, freq=22:

  keys                 the reference state_dict key order (pins the oracle spec / det init)
  step_*               one training step's outputs, losses, gradient norms / heads and BN
                       running stats:
                         *_Adjust: the train_with_adjust.py:96-124 formula (4 losses)
                         *2:       train.py's formula with isadain=True (train.py:89-92:
                                   the re-pass codes from the (codes, features) tuple)
  feats                (*2) the 6 feature scalars [mean, std] x 3 of the step's full pass
  conv_*               a forward of a freshly initialised model in train mode:
                         *2:       target_feature from a second utterance batch
                         *_Adjust: isConvert=True with x_target from a second batch
The reference never travels to the GPU box; only these arrays do.
"""
import os
import sys

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
torch.manual_seed(0)
torch.set_num_threads(8)

B, T, FREQ = 2, 176, 22


def _grads(model):
    out = {}
    for name, p in model.named_parameters():
        g = p.grad if p.grad is not None else torch.zeros_like(p)
        out["gnorm/" + name] = np.array(g.norm().item(), dtype=np.float64)
        out["ghead/" + name] = g.detach().reshape(-1)[:64].numpy().copy()
    return out


def _bn_stats(model):
    return {"bn/" + k: v.detach().numpy().copy() for k, v in model.state_dict().items()
            if "running_" in k or "num_batches_tracked" in k}


def _model(name):
    mod = __import__(f"factory.{name}", fromlist=[name])
    # factory/MetaPool_Adjust.py:250 names its class ``MetaPool`` (so train_with_adjust.py's
    # getattr(module, model_name) lookup cannot reach it); the class is what is recorded
    cls = getattr(mod, name, None) or getattr(mod, name.split("_")[0])
    m = cls(44, 256, 512, FREQ)
    det_init_(m)
    return m.train()


def make(name):
    x, e = det_inputs(B, T)
    x2, e2 = det_inputs(B, T, seed=4321)
    xt, et, x2t, e2t = map(torch.from_numpy, (x, e, x2, e2))
    m = _model(name)
    rec = {"x": x, "emb": e, "x2": x2, "emb2": e2, "T": np.array(T), "freq": np.array(FREQ),
           "keys": np.array(list(m.state_dict().keys()))}
    if name.endswith("_Adjust"):
        emb_adj, x_id, x_psnt, code_real = m(xt, et, et)
        l_id = F.mse_loss(xt, x_id.squeeze())
        l_psnt = F.mse_loss(xt, x_psnt.squeeze())
        code_re = m(x_psnt, et, None)
        l_cd = F.l1_loss(code_real, code_re)
        l_ad = F.l1_loss(emb_adj, et)
        losses = (l_id, l_psnt, l_cd, l_ad)
        rec["step_emb_adj"] = emb_adj.detach().numpy()
    else:
        x_id, x_psnt, code_real = m(xt, et, et)
        l_id = F.mse_loss(xt, x_id.squeeze())
        l_psnt = F.mse_loss(xt, x_psnt.squeeze())
        code_re, _ = m(x_psnt, et, None)
        l_cd = F.l1_loss(code_real, code_re)
        losses = (l_id, l_psnt, l_cd)
    loss = sum(losses)
    m.zero_grad()
    loss.backward()
    rec.update({"step_mel": x_id.detach().numpy(), "step_mel_psnt": x_psnt.detach().numpy(),
                "step_codes": code_real.detach().numpy(), "step_codes_re": code_re.detach().numpy(),
                "step_losses": np.array([v.item() for v in losses], dtype=np.float64)})
    rec.update({"step_" + k: v for k, v in _grads(m).items()})
    rec.update({"step_" + k: v for k, v in _bn_stats(m).items()})

    m = _model(name)
    with torch.no_grad():
        if name.endswith("_Adjust"):
            c_adj, mel, psnt, codes = m(xt, et, e2t, isConvert=True, x_target=x2t)
            rec["conv_emb_adj"] = c_adj.numpy()
        else:
            _, tf = m.encoder(x2t, e2t)
            rec["conv_target_feature"] = np.array([[float(a), float(b)] for a, b in tf])
            mel, psnt, codes = m(xt, et, e2t, target_feature=tf)
    rec.update({"conv_mel": mel.numpy(), "conv_mel_psnt": psnt.numpy(), "conv_codes": codes.numpy()})
    if not name.endswith("_Adjust"):
        m = _model(name)
        with torch.no_grad():
            _, feats = m(xt, et, None)
        rec["feats"] = np.array([[float(a), float(b)] for a, b in feats])
    path = os.path.join(HERE, f"variant_{name}.npz")
    np.savez_compressed(path, **rec)
    print(name, path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    for n in sys.argv[1:] or ["AutoVC2", "AutoVC_Adjust", "MetaConv2", "MetaPool2", "MetaConv_Adjust",
                              "MetaPool_Adjust"]:
        make(n)
