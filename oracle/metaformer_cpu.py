"""ORACLE (test infrastructure only) — CPU restatement of MetaConv / MetaPool.

Restates /root/reference/factory/MetaConv.py, factory/MetaPool.py and
factory/MLPMixer.py as functions of a state_dict with the reference's keys.
Only tests/, smoke() and bench.py's cpu_baseline leg may import it.

Anchors:
  MetaBlock (conv mixer)   MetaConv.py:8-76     forward :64-76
  Pooling mixer            MetaPool.py:7-15     (AvgPool1d(3,1,1,count_include_pad=False) - x)
  Encoder                  MetaConv.py:79-132   (PatchEmbed 336->512, 3 blocks, output_conv, MLP)
  Decoder                  MetaConv.py:135-179  (time axis as channels, crop_len 344)
  MLPMixer                 MLPMixer.py:58-92    (Rearrange b c (h p1) (w p2) -> b (h w) (p1 p2 c))
  GroupNorm(1 group)       Norm.py:53-60
"""
from __future__ import annotations

from collections import OrderedDict

import torch
import torch.nn.functional as F

from .autovc_cpu import _bn, _conv_bn, batch_norm, conv_bn, expand_codes, extract_codes, postnet, postnet_spec

LN_EPS = 1e-5
GN_EPS = 1e-5


# --------------------------------------------------------------------------- spec
def _norm(spec, pre, c):
    spec[f"{pre}.weight"] = (c,)
    spec[f"{pre}.bias"] = (c,)


def mlp_spec(spec, pre, image, patch, dim, out_dim, channels=1, expansion=4, k=5):
    npatch = (image // patch) ** 2
    spec[f"{pre}.1.weight"] = (dim, patch * patch * channels)
    spec[f"{pre}.1.bias"] = (dim,)
    spec[f"{pre}.2.0.fn.0.weight"] = (npatch * expansion, npatch, 1)
    spec[f"{pre}.2.0.fn.0.bias"] = (npatch * expansion,)
    spec[f"{pre}.2.0.fn.3.weight"] = (npatch, npatch * expansion, 1)
    spec[f"{pre}.2.0.fn.3.bias"] = (npatch,)
    _norm(spec, f"{pre}.2.0.norm", dim)
    spec[f"{pre}.2.1.fn.0.weight"] = (dim * expansion, dim)
    spec[f"{pre}.2.1.fn.0.bias"] = (dim * expansion,)
    spec[f"{pre}.2.1.fn.3.weight"] = (dim, dim * expansion)
    spec[f"{pre}.2.1.fn.3.bias"] = (dim,)
    _norm(spec, f"{pre}.2.1.norm", dim)
    spec[f"{pre}.3.weight"] = (out_dim, npatch, k)
    spec[f"{pre}.3.bias"] = (out_dim,)


def metablock_spec(spec, pre, pool, dim=512, crop_len=176, out_dim_neck=88, patch=8):
    _norm(spec, f"{pre}.norm1", dim)
    if not pool:
        _conv_bn(spec, f"{pre}.token_mixer", 512, 512)
    _norm(spec, f"{pre}.norm2", crop_len)
    _conv_bn(spec, f"{pre}.conv_1", 512, crop_len)
    mlp_spec(spec, f"{pre}.mlp", crop_len, patch, crop_len, out_dim_neck)
    _conv_bn(spec, f"{pre}.conv_2", out_dim_neck, 512)


def metaformer_spec(pool: bool, dim_neck=44) -> "OrderedDict[str, tuple]":
    s = OrderedDict()
    s["encoder.embding.proj.weight"] = (512, 336, 5)
    s["encoder.embding.proj.bias"] = (512,)
    for i in range(3):
        metablock_spec(s, f"encoder.metablock.{i}", pool)
    _conv_bn(s, "encoder.output_conv", 512, 176)
    mlp_spec(s, "encoder.mlp", 176, 16, 176, 2 * dim_neck)
    s["decoder.embding.proj.weight"] = (512, 176, 5)
    s["decoder.embding.proj.bias"] = (512,)
    metablock_spec(s, "decoder.metablock.0", pool, crop_len=344, patch=8, out_dim_neck=88)
    _conv_bn(s, "decoder.output_conv_1", 512, 344)
    mlp_spec(s, "decoder.mlp", 344, 8, 344, 88)
    _conv_bn(s, "decoder.output_conv_2", 344, 176)
    s["decoder.linear_projection.linear_layer.weight"] = (80, 88)
    s["decoder.linear_projection.linear_layer.bias"] = (80,)
    postnet_spec(s)
    return s


def metaconv_spec(dim_neck=44, dim_emb=256, dim_pre=512):
    return metaformer_spec(False, dim_neck)


def metapool_spec(dim_neck=44, dim_emb=256, dim_pre=512):
    return metaformer_spec(True, dim_neck)


# --------------------------------------------------------------------------- blocks
def mlp_mixer(x, sd, pre, patch):
    """MLPMixer.py:58-92 with depth=1, dropout 0, expansion 4."""
    B, C, Hh, Ww = x.shape
    h, w = Hh // patch, Ww // patch
    x = x.reshape(B, C, h, patch, w, patch).permute(0, 2, 4, 3, 5, 1).reshape(B, h * w, patch * patch * C)
    x = F.linear(x, sd[f"{pre}.1.weight"], sd[f"{pre}.1.bias"])
    dim = x.shape[-1]
    y = F.layer_norm(x, (dim,), sd[f"{pre}.2.0.norm.weight"], sd[f"{pre}.2.0.norm.bias"], LN_EPS)
    y = F.conv1d(y, sd[f"{pre}.2.0.fn.0.weight"], sd[f"{pre}.2.0.fn.0.bias"])
    y = F.conv1d(F.gelu(y), sd[f"{pre}.2.0.fn.3.weight"], sd[f"{pre}.2.0.fn.3.bias"])
    x = x + y
    y = F.layer_norm(x, (dim,), sd[f"{pre}.2.1.norm.weight"], sd[f"{pre}.2.1.norm.bias"], LN_EPS)
    y = F.linear(y, sd[f"{pre}.2.1.fn.0.weight"], sd[f"{pre}.2.1.fn.0.bias"])
    y = F.linear(F.gelu(y), sd[f"{pre}.2.1.fn.3.weight"], sd[f"{pre}.2.1.fn.3.bias"])
    x = x + y
    return F.conv1d(x, sd[f"{pre}.3.weight"], sd[f"{pre}.3.bias"], padding=2)


def group_norm1(x, sd, pre):
    return F.group_norm(x, 1, sd[f"{pre}.weight"], sd[f"{pre}.bias"], GN_EPS)


def pooling_mixer(x):
    return F.avg_pool1d(x, 3, 1, 1, count_include_pad=False) - x


def metablock(x, sd, pre, pool, patch, training):
    """MetaConv.py:64-76 / MetaPool.py:63-77."""
    y = group_norm1(x, sd, f"{pre}.norm1")
    if pool:
        y = pooling_mixer(y)
    else:
        y = F.relu(conv_bn(y, sd, f"{pre}.token_mixer", training))
    x = x + y
    a = F.relu(conv_bn(x, sd, f"{pre}.conv_1", training))
    m = mlp_mixer(group_norm1(a, sd, f"{pre}.norm2").unsqueeze(1), sd, f"{pre}.mlp", patch)
    return x + F.relu(conv_bn(m, sd, f"{pre}.conv_2", training))


def encoder(sd, x, c_org, dim_neck, freq, training, pool):
    x = x.squeeze(1).transpose(2, 1)
    c = c_org.unsqueeze(-1).expand(-1, -1, x.size(-1))
    h = torch.cat((x, c), dim=1)
    h = F.conv1d(h, sd["encoder.embding.proj.weight"], sd["encoder.embding.proj.bias"], padding=2)
    for i in range(3):
        h = metablock(h, sd, f"encoder.metablock.{i}", pool, 8, training)
    h = F.relu(conv_bn(h, sd, "encoder.output_conv", training))
    h = mlp_mixer(h.unsqueeze(1), sd, "encoder.mlp", 16)
    return extract_codes(h.transpose(1, 2), dim_neck, freq)


def decoder(sd, x, training, pool):
    h = F.conv1d(x, sd["decoder.embding.proj.weight"], sd["decoder.embding.proj.bias"], padding=2)
    h = metablock(h, sd, "decoder.metablock.0", pool, 8, training)
    h = F.relu(conv_bn(h, sd, "decoder.output_conv_1", training))
    h = mlp_mixer(h.unsqueeze(1), sd, "decoder.mlp", 8)
    h = F.relu(conv_bn(h.transpose(2, 1), sd, "decoder.output_conv_2", training))
    return F.linear(h, sd["decoder.linear_projection.linear_layer.weight"],
                    sd["decoder.linear_projection.linear_layer.bias"])


def metaformer_forward(sd, x, c_org, c_trg, dim_neck=44, freq=22, training=True, pool=False):
    """MetaConv.forward (MetaConv.py:254-274) / MetaPool.forward (MetaPool.py:256-276)."""
    codes = encoder(sd, x, c_org, dim_neck, freq, training, pool)
    if c_trg is None:
        return torch.cat(codes, dim=-1)
    enc_out = expand_codes(codes, x.size(1), c_trg)
    mel = decoder(sd, enc_out, training, pool)
    psnt = postnet(sd, mel.transpose(2, 1), training)
    mel_psnt = mel + psnt.transpose(2, 1)
    return mel.unsqueeze(1), mel_psnt.unsqueeze(1), torch.cat(codes, dim=-1)


def metaconv_forward(sd, x, c_org, c_trg, **kw):
    return metaformer_forward(sd, x, c_org, c_trg, pool=False, **kw)


def metapool_forward(sd, x, c_org, c_trg, **kw):
    return metaformer_forward(sd, x, c_org, c_trg, pool=True, **kw)
