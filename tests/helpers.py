"""Shared comparison helpers for the GPU parity tests (SURVEY.md §8(c) bars)."""
import numpy as np
import torch


def rel_inf(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)


def grad_mismatches(model, g, tol=1e-2, head_tol=1e-2,
                    bn_fed_bias=lambda n: "conv.bias" in n and "postnet.convolutions.4" not in n):
    """Per-parameter check against the golden gradient norm (rel <= tol) and first-64-element
    head (max abs error <= head_tol * max(max|head|, rms of the whole golden tensor)): a head
    whose 64 elements happen to be far below the tensor's typical magnitude is held to the
    tensor's scale, not to its own (fp32 reassociation moves every element by ~1e-7 x rms).
    Parameters whose true gradient is analytically zero (conv biases feeding a training-mode
    BatchNorm; `bn_fed_bias`) get an absolute floor only: their golden values are fp32
    rounding noise."""
    bad = {}
    for name, p in model.named_parameters():
        ref_n = float(g["gnorm/" + name])
        got = p.grad.detach().cpu().double()
        head = g["ghead/" + name].astype(np.float64)
        err = np.abs(got.reshape(-1)[:64].numpy() - head).max()
        if bn_fed_bias(name):
            ok = err < 1e-6 + head_tol * np.abs(head).max()
        else:
            scale = max(np.abs(head).max(), ref_n / np.sqrt(max(p.numel(), 1)), 1e-6)
            ok = abs(got.norm().item() - ref_n) <= tol * ref_n + 1e-6 and err <= head_tol * scale
        if not ok:
            bad[name] = (got.norm().item(), ref_n, err)
    return bad


def bn_state_mismatches(model, g):
    bad = []
    for k, v in model.state_dict().items():
        if "running_" in k or "num_batches" in k:
            if not np.allclose(v.detach().cpu().numpy(), g["bn/" + k], rtol=1e-4, atol=1e-6):
                bad.append(k)
    return bad


def to_dev(g, dev, *keys):
    return [torch.from_numpy(g[k]).to(dev) for k in keys]
