"""ORACLE (test infrastructure only) — CPU restatement of the Discriminator and the
two-model step of train_with_discriminator.py.

Anchors:
  Discriminator          factory/Discriminator.py:4-29 (conv k3 no pad, LeakyReLU 0.01, BN, Linear 1628, Sigmoid)
  discriminator_loss     train_with_discriminator.py:58-61
  step                   train_with_discriminator.py:90-111 (ONE loss for G and D, both Adams step)
"""
from __future__ import annotations

from collections import OrderedDict

import torch
import torch.nn.functional as F

from .autovc_cpu import OracleSolver, _bn, autovc_forward, autovc_spec, batch_norm, make_state, params_of, step_losses


def disc_spec(crop_len=176, dim_neck=44) -> "OrderedDict[str, tuple]":
    s = OrderedDict()
    s["conv1.weight"] = (2 * dim_neck, crop_len, 3)
    s["conv1.bias"] = (2 * dim_neck,)
    s["conv2.weight"] = (dim_neck, 2 * dim_neck, 3)
    s["conv2.bias"] = (dim_neck,)
    s["conv3.weight"] = (dim_neck // 2, dim_neck, 3)
    s["conv3.bias"] = (dim_neck // 2,)
    _bn(s, "bn1", dim_neck)
    _bn(s, "bn2", dim_neck // 2)
    s["dense1.weight"] = (1, 1628)
    s["dense1.bias"] = (1,)
    return s


def disc_forward(sd, x, training=True):
    h = F.leaky_relu(F.conv1d(x, sd["conv1.weight"], sd["conv1.bias"]), 0.01)
    h = F.leaky_relu(F.conv1d(h, sd["conv2.weight"], sd["conv2.bias"]), 0.01)
    h = batch_norm(h, sd, "bn1", training)
    h = F.leaky_relu(F.conv1d(h, sd["conv3.weight"], sd["conv3.bias"]), 0.01)
    h = batch_norm(h, sd, "bn2", training)
    h = h.flatten(1)
    return torch.sigmoid(F.linear(h, sd["dense1.weight"], sd["dense1.bias"]))


def discriminator_loss(real, fake):
    return F.binary_cross_entropy(real, torch.ones_like(real)) + F.binary_cross_entropy(fake, torch.zeros_like(fake))


class OracleGANSolver(OracleSolver):
    def __init__(self, lr=1e-4, **kw):
        super().__init__(autovc_spec, autovc_forward, lr=lr, **kw)
        self.dsd = make_state(disc_spec())
        self.dopt = torch.optim.Adam(params_of(self.dsd), lr)

    def step(self, x, emb):
        losses, g, outs = step_losses(self.forward, x, emb)
        d = discriminator_loss(disc_forward(self.dsd, x), disc_forward(self.dsd, outs[1].squeeze()))
        total = g + d
        self.opt.zero_grad()
        self.dopt.zero_grad()
        total.backward()
        self.opt.step()
        self.dopt.step()
        return [l.item() for l in losses] + [d.item()]
