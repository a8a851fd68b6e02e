"""Closed-form deterministic parameter initialiser.

Goldens are generated from the reference modules in the survey container and the
parity tests run on a GPU box that never sees the reference, so both sides need
the *same* weights without shipping a 114 MB checkpoint.  This initialiser is a
pure function of the state_dict layout (key order, key names and shapes), which
the build keeps identical to the reference (``factory/AutoVC.py:182-211``,
SURVEY.md §8(b)).

For the k-th state_dict entry and flat element index n::

    u = splitmix64((k << 40) ^ n) >> 40          # 24-bit integer
    w = bound_k * (2 * u / 2**24 - 1)            # float64, rounded once to fp32

* matrices / conv kernels (ndim >= 2): Xavier bound sqrt(6 / (fan_in + fan_out))
* biases with a >=2-D sibling weight: 1 / sqrt(fan_in of that weight)
* 1-D ``weight`` without a >=2-D sibling (BatchNorm / GroupNorm / LayerNorm γ): 1
* their ``bias`` (β): 0; ``running_mean``: 0; ``running_var``: 1;
  ``num_batches_tracked``: 0
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def uniform24(k: int, n: int) -> np.ndarray:
    """24-bit integers for tensor index k, elements 0..n-1 (as float64 in [0, 2^24))."""
    idx = np.arange(n, dtype=np.uint64)
    key = np.uint64(k) << np.uint64(40)
    return (splitmix64(idx ^ key) >> np.uint64(40)).astype(np.float64)


def _sibling_weight(key: str, shapes: "OrderedDict[str, tuple]"):
    if key.endswith(".bias"):
        cand = key[: -len("bias")] + "weight"
    elif ".bias_ih" in key or key.split(".")[-1].startswith("bias_ih"):
        cand = key.replace("bias_ih", "weight_ih")
    elif key.split(".")[-1].startswith("bias_hh"):
        cand = key.replace("bias_hh", "weight_hh")
    else:
        return None
    return shapes.get(cand)


def det_values(key: str, k: int, shape: tuple, shapes) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    last = key.split(".")[-1]
    if last == "num_batches_tracked":
        return np.zeros(shape, dtype=np.int64)
    if last == "running_mean":
        return np.zeros(shape, dtype=np.float32)
    if last == "running_var":
        return np.ones(shape, dtype=np.float32)
    if len(shape) >= 2:
        rf = int(np.prod(shape[2:])) if len(shape) > 2 else 1
        fan_in, fan_out = shape[1] * rf, shape[0] * rf
        bound = math.sqrt(6.0 / (fan_in + fan_out))
    else:
        sib = _sibling_weight(key, shapes)
        if sib is not None and len(sib) >= 2:
            rf = int(np.prod(sib[2:])) if len(sib) > 2 else 1
            bound = 1.0 / math.sqrt(sib[1] * rf)
        elif last.startswith("weight"):
            return np.ones(shape, dtype=np.float32)
        else:
            return np.zeros(shape, dtype=np.float32)
    u = uniform24(k, n)
    w = bound * (2.0 * u / float(1 << 24) - 1.0)
    return w.astype(np.float32).reshape(shape)


def det_state_dict(template) -> "OrderedDict[str, np.ndarray]":
    """Deterministic values for every entry of a state_dict-like mapping of tensors/arrays."""
    shapes = OrderedDict((k, tuple(v.shape)) for k, v in template.items())
    out = OrderedDict()
    for k, (key, shape) in enumerate(shapes.items()):
        out[key] = det_values(key, k, shape, shapes)
    return out


def det_init_(module) -> None:
    """Overwrite a module's parameters and buffers in place (any device)."""
    import torch

    sd = module.state_dict()
    vals = det_state_dict(sd)
    with torch.no_grad():
        for key, t in sd.items():
            t.copy_(torch.from_numpy(vals[key]).to(t.device, t.dtype))


def det_inputs(batch: int, T: int, dim_emb: int = 256, seed: int = 1234):
    """Deterministic log10-mel-like input (B,T,80) in [-5, 2] and unit-norm speaker
    embeddings (B,dim_emb), matching SURVEY.md §8(d)'s value ranges."""
    u = uniform24(0xA0000 + seed, batch * T * 80) / float(1 << 24)
    x = (-5.0 + 7.0 * u).reshape(batch, T, 80).astype(np.float32)
    e = uniform24(0xB0000 + seed, batch * dim_emb) / float(1 << 24) - 0.5
    e = e.reshape(batch, dim_emb)
    e = e / np.linalg.norm(e, axis=1, keepdims=True)
    return x, e.astype(np.float32)


def det_melgan_state(shapes, gain=(0.7, 1.2)) -> "OrderedDict[str, np.ndarray]":
    """Closed-form weights for the MelGAN generator (melgan/modules.py:88-131) from its
    state_dict (key, shape) list: weight_v as any >= 2-D weight (Xavier bound), weight_g uniform
    in [gain) (positive: each output channel's weight then has that norm; (0.7, 1.2) keeps the 17
    layers' output unsaturated, max |audio| 0.75, std 0.16), bias 1/sqrt(fan_in of
    the sibling weight_v).  Same splitmix64 stream as det_values, keyed by entry index."""
    shapes = OrderedDict((k, tuple(s)) for k, s in shapes)
    out = OrderedDict()
    for k, (key, shape) in enumerate(shapes.items()):
        n = int(np.prod(shape))
        u = uniform24(k, n) / float(1 << 24)
        if key.endswith(".weight_g"):
            w = gain[0] + (gain[1] - gain[0]) * u
        elif key.endswith(".bias"):
            v = shapes[key[: -len("bias")] + "weight_v"]
            fan_in = v[1] * int(np.prod(v[2:]))
            w = (2.0 * u - 1.0) / math.sqrt(fan_in)
        else:
            w = det_values(key, k, shape, shapes).reshape(-1).astype(np.float64)
        out[key] = w.astype(np.float32).reshape(shape)
    return out


def det_mel(batch: int, C: int, T: int, seed: int = 4321):
    """Deterministic (B, C, T) log10-mel-like vocoder input in [-5, 2] (the Converter's range)."""
    u = uniform24(0xC0000 + seed, batch * C * T) / float(1 << 24)
    return (-5.0 + 7.0 * u).reshape(batch, C, T).astype(np.float32)
