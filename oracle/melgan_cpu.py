"""ORACLE (test infrastructure only) — CPU restatement of the MelGAN vocoder generator.

Only ``tests/`` may import this module, as the checker.  The product path
(autoformer_amd/melgan.py, HIP kernels) never imports it.

It restates /root/reference/melgan/modules.py:88-131 (`Generator(input_size, ngf,
n_residual_layers)`, with `ResnetBlock` :72-86 and the weight-normed convs :18-23) as a pure
function of a state_dict with the reference's keys, on PyTorch CPU ops: weight norm written out
(w = g v / ||v||, norm over every dim but dim 0 -- torch.nn.utils.weight_norm's default, which
for ConvTranspose1d's [in][out][k] weight is per INPUT channel), F.pad(mode="reflect"),
F.leaky_relu(0.2), F.conv1d / F.conv_transpose1d, tanh.  Pinned against fixtures generated
from the reference module itself (tests/golden/make_melgan_goldens.py, melgan_G.npz;
tests/test_melgan.py).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

RATIOS = (8, 8, 2, 2)  # modules.py:91
SLOPE = 0.2            # modules.py:75,78,108,123


def wn_weight(sd, prefix):
    """modules.py:18-23 weight_norm(dim=0): g * v / ||v|| (norm over all dims but 0)."""
    v, g = sd[prefix + ".weight_v"].float(), sd[prefix + ".weight_g"].float()
    n = v.reshape(v.shape[0], -1).norm(dim=1).reshape((-1,) + (1,) * (v.dim() - 1))
    return g * v / n


def resnet_block(sd, prefix, x, dilation):
    """modules.py:72-86: shortcut(x) + block(x)."""
    h = F.leaky_relu(x, SLOPE)
    h = F.pad(h, (dilation, dilation), mode="reflect")
    h = F.conv1d(h, wn_weight(sd, prefix + ".block.2"), sd[prefix + ".block.2.bias"], dilation=dilation)
    h = F.leaky_relu(h, SLOPE)
    h = F.conv1d(h, wn_weight(sd, prefix + ".block.4"), sd[prefix + ".block.4.bias"])
    s = F.conv1d(x, wn_weight(sd, prefix + ".shortcut"), sd[prefix + ".shortcut.bias"])
    return s + h


def generator(sd, mel, n_residual_layers=3):
    """modules.py:88-131 forward: (B, input_size, T) -> (B, 1, T * 256)."""
    x = F.pad(mel.float(), (3, 3), mode="reflect")                       # model.0
    x = F.conv1d(x, wn_weight(sd, "model.1"), sd["model.1.bias"])       # model.1
    i = 2
    for r in RATIOS:                                                     # :97-118
        x = F.leaky_relu(x, SLOPE)                                       # model.i
        x = F.conv_transpose1d(x, wn_weight(sd, f"model.{i + 1}"), sd[f"model.{i + 1}.bias"], stride=r,
                               padding=r // 2 + r % 2, output_padding=r % 2)
        i += 2
        for j in range(n_residual_layers):
            x = resnet_block(sd, f"model.{i}", x, 3 ** j)
            i += 1
    x = F.leaky_relu(x, SLOPE)                                           # :122-127
    x = F.pad(x, (3, 3), mode="reflect")
    x = F.conv1d(x, wn_weight(sd, f"model.{i + 2}"), sd[f"model.{i + 2}.bias"])
    return torch.tanh(x)
