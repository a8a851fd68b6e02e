"""ORACLE (test infrastructure only) — CPU restatement of the AdaIN ("2") and
speaker-embedding-adjust ("_Adjust") model variants.

Only tests/ may import this module, and only as the checker.  It composes the AutoVC /
MetaConv / MetaPool restatements (oracle/autovc_cpu.py, oracle/metaformer_cpu.py) with the
variant pieces, as functions of a state_dict with the reference's keys.  Pinned against
goldens produced from the reference modules by tests/golden/make_variant_goldens.py
(tests/test_oracle_goldens.py).

Anchors:
  feature_pre_extract   factory/AutoVC2.py:14-33 (init), :56-61 (forward: conv -> BN, then
                        [x.mean(), x.std()] of the WHOLE tensor, unbiased std)
  AdaIN                 factory/Norm.py:84-91  ((c - c.mean()) / c.std() * std + mu)
  Postnet (AdaIN)       factory/AutoVC2.py:175-201 (after the 5 convs: 3 x (AdaIN, conv 80->80))
  AutoVC2.forward       factory/AutoVC2.py:213-242 (c_trg None and no target_feature -> (codes, features))
  MetaConv2/MetaPool2   factory/MetaConv2.py:86-157, :262-325; factory/MetaPool2.py (same edits)
  Adjust                factory/Adjust.py:7-43 (concat emb, 3 x ReLU(BN(conv5)), LSTM(512, 768, 3),
                        last step, Linear 768->256, L2 normalise)
  *_Adjust.forward      factory/AutoVC_Adjust.py:177-205, MetaConv_Adjust.py:255-279,
                        MetaPool_Adjust.py:258-282
  train_with_adjust     train_with_adjust.py:96-124 (loss = id + id_psnt + cd + l1(emb_adjust, emb))
"""
from __future__ import annotations

from collections import OrderedDict

import torch
import torch.nn.functional as F

from . import autovc_cpu as A
from . import metaformer_cpu as M


# --------------------------------------------------------------------------- specs
def _pre_extract_spec(s, pre="encoder.feature_pre_extract"):
    for i in range(3):
        A._conv_bn(s, f"{pre}.{i}", 80, 80)


def _combine_spec(s, pre="postnet.feature_last_combine"):
    for i in range(3):
        s[f"{pre}.{i}.0.conv.weight"] = (80, 80, 5)
        s[f"{pre}.{i}.0.conv.bias"] = (80,)


def adjust_spec(s, dim_emb=256, dim_cell=768, pre="adjust"):
    for i in range(3):
        A._conv_bn(s, f"{pre}.convolutions.{i}", 80 + dim_emb if i == 0 else 512, 512)
    A._lstm(s, f"{pre}.lstm", 512, dim_cell, 3, False)
    s[f"{pre}.embedding.linear_layer.weight"] = (256, dim_cell)
    s[f"{pre}.embedding.linear_layer.bias"] = (256,)


def _adain_variant(base: "OrderedDict[str, tuple]") -> "OrderedDict[str, tuple]":
    """Insert the pre-extract convs first in the encoder and the combine convs last."""
    s = OrderedDict()
    _pre_extract_spec(s)
    for k, v in base.items():
        s[k] = v
    _combine_spec(s)
    return s


def autovc2_spec():
    return _adain_variant(A.autovc_spec())


def metaconv2_spec():
    return _adain_variant(M.metaconv_spec())


def metapool2_spec():
    return _adain_variant(M.metapool_spec())


def _adjust_variant(base):
    s = OrderedDict(base)
    adjust_spec(s)
    return s


def autovc_adjust_spec():
    return _adjust_variant(A.autovc_spec())


def metaconv_adjust_spec():
    return _adjust_variant(M.metaconv_spec())


def metapool_adjust_spec():
    return _adjust_variant(M.metapool_spec())


SPECS = {
    "AutoVC2": autovc2_spec, "MetaConv2": metaconv2_spec, "MetaPool2": metapool2_spec,
    "AutoVC_Adjust": autovc_adjust_spec, "MetaConv_Adjust": metaconv_adjust_spec,
    "MetaPool_Adjust": metapool_adjust_spec,
}


# --------------------------------------------------------------------------- pieces
def adain(content, mu, std):
    """Norm.py:84-91."""
    return (content - content.mean()) / content.std() * std + mu


def pre_extract(sd, x, training, pre="encoder.feature_pre_extract"):
    """(B, T, 80) or (B, 1, T, 80) -> (B, T, 80) after 3 x conv->BN, plus the features."""
    h = x.squeeze(1).transpose(2, 1)
    feats = []
    for i in range(3):
        h = A.conv_bn(h, sd, f"{pre}.{i}", training)
        feats.append([h.mean(), h.std()])
    return h.transpose(1, 2), feats


def postnet_adain(sd, x, feats, training, pre="postnet"):
    h = A.postnet(sd, x, training, pre)
    for i, f in enumerate(feats):
        h = adain(h, f[0], f[1])
        h = F.conv1d(h, sd[f"{pre}.feature_last_combine.{i}.0.conv.weight"],
                     sd[f"{pre}.feature_last_combine.{i}.0.conv.bias"], padding=2)
    return h


def adjust(sd, x, emb, training, dim_cell=768, pre="adjust"):
    """Adjust.forward (Adjust.py:36-43)."""
    h = x.squeeze(1).transpose(2, 1)
    h = torch.cat((h, emb.unsqueeze(-1).expand(-1, -1, h.size(-1))), dim=1)
    for i in range(3):
        h = F.relu(A.conv_bn(h, sd, f"{pre}.convolutions.{i}", training))
    h = A.lstm(h.transpose(1, 2), sd, f"{pre}.lstm", dim_cell, 3, False, training)[:, -1, :]
    e = F.linear(h, sd[f"{pre}.embedding.linear_layer.weight"], sd[f"{pre}.embedding.linear_layer.bias"])
    return e.div(e.norm(p=2, dim=-1, keepdim=True))


def _family(name):
    if name.startswith("AutoVC"):
        enc = lambda sd, x, c, freq, tr: A.encoder(sd, x, c, 44, freq, tr)  # noqa: E731
        dec = lambda sd, x, tr: A.decoder(sd, x, tr)  # noqa: E731
    else:
        pool = name.startswith("MetaPool")
        enc = lambda sd, x, c, freq, tr: M.encoder(sd, x, c, 44, freq, tr, pool)  # noqa: E731
        dec = lambda sd, x, tr: M.decoder(sd, x, tr, pool)  # noqa: E731
    return enc, dec


# whether forward() runs c_org through Adjust (AutoVC_Adjust.py:179, MetaConv_Adjust.py:256;
# MetaPool_Adjust.py:258-260 does not)
ADJUSTS_ORG = {"AutoVC_Adjust": True, "MetaConv_Adjust": True, "MetaPool_Adjust": False}


# --------------------------------------------------------------------------- forwards
def adain_forward(name, sd, x, c_org, c_trg, target_feature=None, freq=22, training=True):
    """AutoVC2.forward (AutoVC2.py:213-242); MetaConv2 / MetaPool2 likewise."""
    enc, dec = _family(name)
    h, feats = pre_extract(sd, x, training)
    codes = enc(sd, h, c_org, freq, training)
    if c_trg is None and target_feature is None:
        return torch.cat(codes, dim=-1), feats
    enc_out = A.expand_codes(codes, x.size(1) if x.dim() == 3 else x.size(2), c_trg)
    mel = dec(sd, enc_out, training)
    psnt = postnet_adain(sd, mel.transpose(2, 1), target_feature if target_feature is not None else feats,
                         training)
    mel_psnt = mel + psnt.transpose(2, 1)
    return mel.unsqueeze(1), mel_psnt.unsqueeze(1), torch.cat(codes, dim=-1)


def adjust_forward(name, sd, x, c_org, c_trg, isConvert=False, x_target=None, freq=22, training=True):
    """AutoVC_Adjust.forward (AutoVC_Adjust.py:177-205); Meta*_Adjust likewise, except that
    MetaPool_Adjust.py:258-282 never adjusts c_org (it is encoded and returned as given)."""
    enc, dec = _family(name)
    if ADJUSTS_ORG[name]:
        c_org = adjust(sd, x, c_org, training)
    codes = enc(sd, x, c_org, freq, training)
    if c_trg is None:
        return torch.cat(codes, dim=-1)
    elif isConvert:
        c_trg = adjust(sd, x_target, c_trg, training)
    else:
        c_trg = adjust(sd, x, c_trg, training)
    T = x.size(1) if x.dim() == 3 else x.size(2)
    enc_out = A.expand_codes(codes, T, c_trg)
    mel = dec(sd, enc_out, training)
    psnt = A.postnet(sd, mel.transpose(2, 1), training)
    mel_psnt = mel + psnt.transpose(2, 1)
    return c_org, mel.unsqueeze(1), mel_psnt.unsqueeze(1), torch.cat(codes, dim=-1)


def adjust_step_losses(forward, x, emb, lambda_cd=1.0, lambda_ad=1.0):
    """Loss formula of train_with_adjust.Solver.train (train_with_adjust.py:96-124)."""
    emb_adj, x_id, x_id_psnt, code_real = forward(x, emb, emb)
    l_id = F.mse_loss(x, x_id.squeeze())
    l_id_psnt = F.mse_loss(x, x_id_psnt.squeeze())
    code_re = forward(x_id_psnt, emb, None)
    l_cd = F.l1_loss(code_real, code_re)
    l_ad = F.l1_loss(emb_adj, emb)
    total = l_id + l_id_psnt + lambda_cd * l_cd + lambda_ad * l_ad
    return (l_id, l_id_psnt, l_cd, l_ad), total, (emb_adj, x_id, x_id_psnt, code_real, code_re)


def adain_step_losses(forward, x, emb):
    """train.py's step with isadain=True (train.py:89-92, `--use_adain`): the re-pass returns
    (codes, features) and its codes are the first element; the loss formula of train.py:84-96."""
    x_id, x_id_psnt, code_real = forward(x, emb, emb)
    l_id = F.mse_loss(x, x_id.squeeze())
    l_id_psnt = F.mse_loss(x, x_id_psnt.squeeze())
    code_re, _ = forward(x_id_psnt, emb, None)
    l_cd = F.l1_loss(code_real, code_re)
    return (l_id, l_id_psnt, l_cd), l_id + l_id_psnt + l_cd, (x_id, x_id_psnt, code_real, code_re)
