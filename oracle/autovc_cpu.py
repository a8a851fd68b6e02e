"""ORACLE (test infrastructure only) — CPU restatement of the AutoVC training path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / the timed CPU baseline.  The product
path (autoformer_amd) never imports it.

It restates /root/reference/factory/AutoVC.py as pure functions of a state_dict
(the same keys/shapes as the reference) using PyTorch CPU ops
(F.conv1d / F.batch_norm / torch.lstm, which are the ops the reference modules
dispatch to).  It is pinned against the goldens produced from the reference
itself by tests/golden/make_goldens.py (tests/test_oracle_goldens.py).

Reference anchors:
  Encoder      factory/AutoVC.py:18-68   (conv stack :50-51, BiLSTM :54-55, codes :59-66)
  Decoder      factory/AutoVC.py:71-114
  Postnet      factory/AutoVC.py:117-179
  AutoVC       factory/AutoVC.py:182-211
  ConvNorm     factory/Norm.py:4-37      (padding = dilation*(k-1)/2)
  Solver step  train.py:82-99
"""
from __future__ import annotations

from collections import OrderedDict

import torch
import torch.nn.functional as F

BN_MOMENTUM = 0.1
BN_EPS = 1e-5


# --------------------------------------------------------------------------- spec
def _conv_bn(spec, pre, cin, cout, k=5):
    spec[f"{pre}.0.conv.weight"] = (cout, cin, k)
    spec[f"{pre}.0.conv.bias"] = (cout,)
    _bn(spec, f"{pre}.1", cout)


def _bn(spec, pre, c):
    spec[f"{pre}.weight"] = (c,)
    spec[f"{pre}.bias"] = (c,)
    spec[f"{pre}.running_mean"] = (c,)
    spec[f"{pre}.running_var"] = (c,)
    spec[f"{pre}.num_batches_tracked"] = ()


def _lstm(spec, pre, cin, hidden, layers, bidir):
    for layer in range(layers):
        lin = cin if layer == 0 else hidden * (2 if bidir else 1)
        for sfx in (["", "_reverse"] if bidir else [""]):
            spec[f"{pre}.weight_ih_l{layer}{sfx}"] = (4 * hidden, lin)
            spec[f"{pre}.weight_hh_l{layer}{sfx}"] = (4 * hidden, hidden)
            spec[f"{pre}.bias_ih_l{layer}{sfx}"] = (4 * hidden,)
            spec[f"{pre}.bias_hh_l{layer}{sfx}"] = (4 * hidden,)


def postnet_spec(spec, pre="postnet"):
    chans = [80, 512, 512, 512, 512, 80]
    for i in range(5):
        _conv_bn(spec, f"{pre}.convolutions.{i}", chans[i], chans[i + 1])


def autovc_spec(dim_neck=44, dim_emb=256, dim_pre=512) -> "OrderedDict[str, tuple]":
    s = OrderedDict()
    for i in range(3):
        _conv_bn(s, f"encoder.convolutions.{i}", 80 + dim_emb if i == 0 else 512, 512)
    _lstm(s, "encoder.lstm", 512, dim_neck, 2, True)
    _lstm(s, "decoder.lstm1", dim_neck * 2 + dim_emb, dim_pre, 1, False)
    for i in range(3):
        _conv_bn(s, f"decoder.convolutions.{i}", dim_pre, dim_pre)
    _lstm(s, "decoder.lstm2", dim_pre, 1024, 2, False)
    s["decoder.linear_projection.linear_layer.weight"] = (80, 1024)
    s["decoder.linear_projection.linear_layer.bias"] = (80,)
    postnet_spec(s)
    return s


def make_state(spec, values=None, device="cpu"):
    """Tensors for a spec; params (float, not BN buffers) get requires_grad."""
    from autoformer_amd.detinit import det_state_dict

    if values is None:
        values = det_state_dict(OrderedDict((k, torch.empty(v)) for k, v in spec.items()))
    sd = OrderedDict()
    for k, shape in spec.items():
        t = torch.as_tensor(values[k]).clone().to(device)
        if t.is_floating_point() and not any(b in k for b in ("running_mean", "running_var")):
            t.requires_grad_(True)
        sd[k] = t
    return sd


def params_of(sd):
    return [t for t in sd.values() if t.requires_grad]


# --------------------------------------------------------------------------- blocks
def batch_norm(x, sd, pre, training):
    if training:
        sd[f"{pre}.num_batches_tracked"].add_(1)
    return F.batch_norm(x, sd[f"{pre}.running_mean"], sd[f"{pre}.running_var"],
                        sd[f"{pre}.weight"], sd[f"{pre}.bias"], training, BN_MOMENTUM, BN_EPS)


def conv_bn(x, sd, pre, training, pad=None):
    """ConvNorm + BatchNorm1d on (B, C, T) — Norm.py:4-37 (+ nn.BatchNorm1d)."""
    w = sd[f"{pre}.0.conv.weight"]
    if pad is None:
        pad = (w.shape[-1] - 1) // 2
    y = F.conv1d(x, w, sd[f"{pre}.0.conv.bias"], padding=pad)
    return batch_norm(y, sd, f"{pre}.1", training)


def lstm(x, sd, pre, hidden, layers, bidir, training=True):
    """Multi-layer (Bi)LSTM, batch_first, h0=c0=0 (torch.lstm is nn.LSTM's kernel)."""
    params = []
    for layer in range(layers):
        for sfx in (["", "_reverse"] if bidir else [""]):
            for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh"):
                params.append(sd[f"{pre}.{n}_l{layer}{sfx}"])
    nd = 2 if bidir else 1
    h0 = x.new_zeros(layers * nd, x.shape[0], hidden)
    out, _, _ = torch.lstm(x, (h0, h0), params, True, layers, 0.0, training, bidir, True)
    return out


def lstm_loop(x, w_ih, w_hh, b_ih, b_hh, reverse=False):
    """Explicit recurrence (gate order i, f, g, o as in torch.nn.LSTM) — cross-check only."""
    B, T, _ = x.shape
    H = w_hh.shape[1]
    h = x.new_zeros(B, H)
    c = x.new_zeros(B, H)
    outs = [None] * T
    steps = range(T - 1, -1, -1) if reverse else range(T)
    for t in steps:
        g = x[:, t] @ w_ih.t() + b_ih + h @ w_hh.t() + b_hh
        i, f, gg, o = g.chunk(4, dim=1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
        h = torch.sigmoid(o) * torch.tanh(c)
        outs[t] = h
    return torch.stack(outs, 1)


def extract_codes(outputs, dim_neck, freq):
    """AutoVC.py:56-66 — fwd half at the last frame of each segment, bwd half at the first."""
    fwd = outputs[:, :, :dim_neck]
    bwd = outputs[:, :, dim_neck:]
    return [torch.cat((fwd[:, i + freq - 1, :], bwd[:, i, :]), dim=-1)
            for i in range(0, outputs.size(1), freq)]


def encoder(sd, x, c_org, dim_neck, freq, training, pre="encoder"):
    x = x.squeeze(1).transpose(2, 1)
    c = c_org.unsqueeze(-1).expand(-1, -1, x.size(-1))
    h = torch.cat((x, c), dim=1)
    for i in range(3):
        h = F.relu(conv_bn(h, sd, f"{pre}.convolutions.{i}", training))
    h = h.transpose(1, 2)
    out = lstm(h, sd, f"{pre}.lstm", dim_neck, 2, True, training)
    return extract_codes(out, dim_neck, freq)


def decoder(sd, x, training, dim_pre=512, pre="decoder"):
    h = lstm(x, sd, f"{pre}.lstm1", dim_pre, 1, False, training)
    h = h.transpose(1, 2)
    for i in range(3):
        h = F.relu(conv_bn(h, sd, f"{pre}.convolutions.{i}", training))
    h = h.transpose(1, 2)
    h = lstm(h, sd, f"{pre}.lstm2", 1024, 2, False, training)
    return F.linear(h, sd[f"{pre}.linear_projection.linear_layer.weight"],
                    sd[f"{pre}.linear_projection.linear_layer.bias"])


def postnet(sd, x, training, pre="postnet"):
    for i in range(4):
        x = torch.tanh(conv_bn(x, sd, f"{pre}.convolutions.{i}", training))
    return conv_bn(x, sd, f"{pre}.convolutions.4", training)


def expand_codes(codes, T, c_trg):
    """AutoVC.py:197-204."""
    tmp = [code.unsqueeze(1).expand(-1, int(T / len(codes)), -1) for code in codes]
    code_exp = torch.cat(tmp, dim=1)
    return torch.cat((code_exp, c_trg.unsqueeze(1).expand(-1, T, -1)), dim=-1)


def autovc_forward(sd, x, c_org, c_trg, dim_neck=44, freq=22, training=True):
    """AutoVC.forward (AutoVC.py:191-211)."""
    codes = encoder(sd, x, c_org, dim_neck, freq, training)
    if c_trg is None:
        return torch.cat(codes, dim=-1)
    enc_out = expand_codes(codes, x.size(1), c_trg)
    mel = decoder(sd, enc_out, training)
    psnt = postnet(sd, mel.transpose(2, 1), training)
    mel_psnt = mel + psnt.transpose(2, 1)
    return mel.unsqueeze(1), mel_psnt.unsqueeze(1), torch.cat(codes, dim=-1)


# --------------------------------------------------------------------------- solver
def step_losses(forward, x, emb, lambda_cd=1.0):
    """Loss formula of Solver.train (train.py:84-96)."""
    x_id, x_id_psnt, code_real = forward(x, emb, emb)
    l_id = F.mse_loss(x, x_id.squeeze())
    l_id_psnt = F.mse_loss(x, x_id_psnt.squeeze())
    code_re = forward(x_id_psnt, emb, None)
    l_cd = F.l1_loss(code_real, code_re)
    return (l_id, l_id_psnt, l_cd), l_id + l_id_psnt + lambda_cd * l_cd, (x_id, x_id_psnt, code_real, code_re)


class OracleSolver:
    """train.py Solver (train.py:13-132) restated on a functional state_dict."""

    def __init__(self, spec_fn=autovc_spec, forward_fn=autovc_forward, dim_neck=44, freq=22,
                 lr=1e-4, values=None, **fw_kw):
        self.sd = make_state(spec_fn(), values)
        self.freq = freq
        self.dim_neck = dim_neck
        self.forward_fn = forward_fn
        self.fw_kw = fw_kw
        self.opt = torch.optim.Adam(params_of(self.sd), lr)

    def forward(self, x, c_org, c_trg):
        return self.forward_fn(self.sd, x, c_org, c_trg, dim_neck=self.dim_neck, freq=self.freq,
                               training=True, **self.fw_kw)

    def step(self, x, emb):
        losses, total, _ = step_losses(self.forward, x, emb)
        self.opt.zero_grad()
        total.backward()
        self.opt.step()
        return [l.item() for l in losses]
