"""AutoVC (Qian et al., 2019) on MI355X — drop-in for /root/reference/factory/AutoVC.py.

Same constructor ``AutoVC(dim_neck, dim_emb, dim_pre, freq)``, same
``forward(x, c_org, c_trg)`` contract (returns ``(mel (B,1,T,80), mel_postnet (B,1,T,80),
codes (B, T/freq*2*dim_neck))``, or only ``codes`` when ``c_trg is None``) and the same
``state_dict`` keys, so the reference's train.py / train_with_discriminator.py run it
unchanged through their ``importlib`` plugin lookup (train.py:45-47).

Every op runs as a HIP kernel from libautovc_hip.so:
  Encoder  AutoVC.py:18-68  -> enc_conv0 (the speaker half of cat(mel, c_org) folded into a
                               per-(utterance, edge class) GEMM row bias; the conv runs on the 80
                               mel channels, fold.hip), 2x conv_bn (BN statistics + finalize in the
                               conv epilogue), 2 BiLSTM layers (persistent small-H recurrence),
                               code gather
  Decoder  AutoVC.py:71-114 -> lstm1 (input projection folded per code / utterance, persistent
                               recurrence), 3x conv_bn, lstm2 (2 layers: one-launch wavefront
                               forward, persistent backward per layer), linear
  Postnet  AutoVC.py:117-179-> 5x conv_bn (tanh x4, none x1 with the residual add fused)
Activations are frame-major (B*T, C); the reference's (B, C, T) transposes disappear.
"""
import os

import torch
import torch.nn as nn

from .. import kernels as K
from .. import layers as Lyr
from .Norm import ConvNorm, LinearNorm, LSTMParams


# AVC_FOLD=0: the unfolded concat + lstm1 path (A/B and parity diagnostics)
_FOLD = os.environ.get("AVC_FOLD", "1") != "0"


def _conv_bn_block(cin, cout, gain):
    return nn.Sequential(ConvNorm(cin, cout, kernel_size=5, stride=1, padding=2, dilation=1, w_init_gain=gain),
                         nn.BatchNorm1d(cout))


def _frames(x):
    """(B,T,C) or (B,1,T,C) -> contiguous (B*T, C), B, T (AutoVC.py:46 squeeze(1))."""
    if x.dim() == 4:
        x = x.squeeze(1)
    B, T, C = x.shape
    return x.reshape(B * T, C).contiguous(), B, T


class Encoder(nn.Module):
    """Encoder module (AutoVC.py:18-68)."""

    def __init__(self, dim_neck, dim_emb, freq):
        super().__init__()
        self.dim_neck = dim_neck
        self.freq = freq
        self.convolutions = nn.ModuleList(
            [_conv_bn_block(80 + dim_emb if i == 0 else 512, 512, "relu") for i in range(3)])
        self.lstm = LSTMParams(512, dim_neck, 2, batch_first=True, bidirectional=True)
        self._convs = [Lyr.ConvBNCore(s[0].conv, s[1], K.ACT_RELU) for s in self.convolutions]
        self._lstm = [Lyr.LSTMLayerCore(self.lstm, layer) for layer in range(2)]

    def codes_flat(self, x, c_org):
        mel, B, T = _frames(x)
        return self.codes_frames(mel, c_org, B, T)

    def codes_frames(self, mel, c_org, B, T):
        """Frame-major mel (B*T, 80) -> codes (B, T/freq * 2*dim_neck)."""
        if T % self.freq:
            # the reference indexes out_forward[:, i + freq - 1] past T here (AutoVC.py:63)
            raise IndexError(f"len_crop {T} is not a multiple of freq {self.freq}")
        # conv outputs feed only the next conv / the BiLSTM input projection: bf16 storage
        h = Lyr.enc_conv0(self._convs[0], mel, c_org.contiguous(), B, T, out_bf16=True)
        for core in self._convs[1:]:  # each conv output feeds the next conv alone (fuse_prev)
            h = Lyr.conv_bn(core, h, B, T, out_bf16=True, fuse_prev=True)
        h = Lyr.lstm(self.lstm, self._lstm, h, B, T)
        return Lyr.codes(h, B, T, self.dim_neck, self.freq)

    def forward(self, x, c_org):
        K.require_device(x, c_org)
        return list(self.codes_flat(x, c_org).split(2 * self.dim_neck, dim=-1))


class Decoder(nn.Module):
    """Decoder module (AutoVC.py:71-114)."""

    def __init__(self, dim_neck, dim_emb, dim_pre):
        super().__init__()
        self.lstm1 = LSTMParams(dim_neck * 2 + dim_emb, dim_pre, 1, batch_first=True)
        self.convolutions = nn.ModuleList([_conv_bn_block(dim_pre, dim_pre, "relu") for _ in range(3)])
        self.lstm2 = LSTMParams(dim_pre, 1024, 2, batch_first=True)
        self.linear_projection = LinearNorm(1024, 80)
        self._lstm1 = [Lyr.LSTMLayerCore(self.lstm1, 0)]
        self._convs = [Lyr.ConvBNCore(s[0].conv, s[1], K.ACT_RELU) for s in self.convolutions]
        self._lstm2 = [Lyr.LSTMLayerCore(self.lstm2, layer) for layer in range(2)]
        self._lin = Lyr.PackCache()

    def frames(self, x, B, T):
        return self._after_lstm1(Lyr.lstm(self.lstm1, self._lstm1, x, B, T), B, T)

    def frames_codes(self, codes, c_trg, B, T, nc, cd, hook=None):
        """frames(cat(code expansion, c_trg broadcast)) with lstm1's input projection folded per
        code and per utterance (layers._LSTM1FoldFn); hook: see decode()."""
        h = Lyr.lstm1_folded(self.lstm1, self._lstm1[0], codes, c_trg, B, T, nc, cd, hook)
        return self._after_lstm1(h, B, T)

    def _after_lstm1(self, h, B, T):
        for core in self._convs:  # (lstm1's output carries no BN link: fuse_prev is a no-op there)
            h = Lyr.conv_bn(core, h, B, T, out_bf16=True, fuse_prev=True)
        h = Lyr.lstm(self.lstm2, self._lstm2, h, B, T)
        lin = self.linear_projection.linear_layer
        return Lyr.linear(h, lin.weight, lin.bias, self._lin)

    def forward(self, x):
        K.require_device(x)
        xf, B, T = _frames(x)
        return self.frames(xf, B, T).view(B, T, -1)


class Postnet(nn.Module):
    """Postnet: five 1-d convolutions with 512 channels and kernel size 5 (AutoVC.py:117-179)."""

    def __init__(self):
        super().__init__()
        self.convolutions = nn.ModuleList()
        self.convolutions.append(_conv_bn_block(80, 512, "tanh"))
        for _ in range(1, 5 - 1):
            self.convolutions.append(_conv_bn_block(512, 512, "tanh"))
        self.convolutions.append(_conv_bn_block(512, 80, "linear"))
        self._convs = [Lyr.ConvBNCore(s[0].conv, s[1], K.ACT_TANH) for s in self.convolutions[:-1]]
        self._convs.append(Lyr.ConvBNCore(self.convolutions[-1][0].conv, self.convolutions[-1][1], K.ACT_NONE))

    def frames(self, mel, B, T, residual=None):
        h = mel
        for core in self._convs[:-1]:
            h = Lyr.conv_bn(core, h, B, T, out_bf16=True, fuse_prev=True)
        return Lyr.conv_bn(self._convs[-1], h, B, T, residual=residual, fuse_prev=True)

    def forward(self, x):
        """Reference layout (B, 80, T) in and out."""
        K.require_device(x)
        B, C, T = x.shape
        xf = Lyr.bct_to_frames(x)
        return Lyr.frames_to_bct(self.frames(xf, B, T), B, T)


class AutoVC(nn.Module):
    """Generator network (AutoVC.py:182-211)."""

    def __init__(self, dim_neck, dim_emb, dim_pre, freq):
        super().__init__()
        self.encoder = Encoder(dim_neck, dim_emb, freq)
        self.decoder = Decoder(dim_neck, dim_emb, dim_pre)
        self.postnet = Postnet()
        self.dim_neck = dim_neck

    def forward(self, x, c_org, c_trg):
        K.require_device(x, c_org, c_trg)
        codes = self.encoder.codes_flat(x, c_org)
        if c_trg is None:
            return codes
        return decode(self, x, codes, c_trg)


def decode(model, x, codes, c_trg, features=None):
    """Code expansion + c_trg concat, decoder, postnet (+ residual) (AutoVC.py:197-211);
    shared by every model family and variant.  `features`: the AdaIN postnet's statistics
    (AutoVC2.py:231-237)."""
    xs = x.squeeze(1) if x.dim() == 4 else x
    B, T = xs.shape[0], xs.shape[1]
    cd = 2 * model.dim_neck
    nc = codes.shape[1] // cd
    # fires once the backward has produced every decoder / postnet gradient
    hook = getattr(model, "_decoder_bwd_done", None)
    if hasattr(model.decoder, "frames_codes") and _FOLD:
        mel = model.decoder.frames_codes(codes, c_trg.contiguous(), B, T, nc, cd, hook)
    else:
        enc_out = Lyr.dec_concat(codes, c_trg.contiguous(), B, T, nc, cd)
        if hook is not None and enc_out.requires_grad:
            enc_out.register_hook(lambda g: hook())
        mel = model.decoder.frames(enc_out, B, T)
    if features is None:
        mel_postnet = model.postnet.frames(mel, B, T, residual=mel)
    else:
        mel_postnet = model.postnet.frames(mel, B, T, features, residual=mel)
    return mel.view(B, 1, T, -1), mel_postnet.view(B, 1, T, -1), codes
