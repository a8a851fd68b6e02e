"""MelGAN vocoder generator on the HIP path (the conversion path's mel ->
waveform step, reference melgan/modules.py:88-131 `Generator`, melgan/interface.py:23-53
`MelVocoder.inverse`, called by util/evaluate.py:96-98 `get_wavs`).

Drop-in: `Generator(input_size, ngf, n_residual_layers)` builds the reference's module tree
(ReflectionPad1d / weight-normed Conv1d / LeakyReLU / weight-normed ConvTranspose1d /
ResnetBlock, modules.py:72-86,88-131) only as the parameter container, so `state_dict()` keys
and shapes are the reference's (`model.1.weight_g`, `model.4.block.2.weight_v`,
`model.21.shortcut.bias`, ...) and a reference checkpoint loads unchanged.  `forward(mel)`
never runs those submodules: it runs frame-major HIP kernels (melgan.hip + avc_gemm):

  conv_in     mg_gather (reflect 3, 7 taps) -> GEMM 80*7 -> 512
  upsample r  LeakyReLU twin -> ONE GEMM over the zero-padded 3-tap window, N = r*Cout
              (polyphase ConvTranspose1d, avc_mg_wn_pack): its [B*L][r*Cout] output is the
              upsampled [B*L*r][Cout] sequence
  ResnetBlock mg_gather (reflect d, dilation d = 1, 3, 9, LeakyReLU) -> GEMM 3C -> C ->
              LeakyReLU twin; shortcut GEMM C -> C, then the 1x1 GEMM accumulated onto it
  conv_out    mg_conv_out (LeakyReLU, reflect 3, 7 taps, 32 -> 1, tanh)

Weight norm (g v / ||v||) is folded into the packed GEMM operands once per parameter version
(inference weights do not change between calls).  There is no CPU or torch fallback: the
kernels raise on host tensors.
"""
from __future__ import annotations

import warnings

import numpy as np
import torch
import torch.nn as nn

from . import _lib as L
from . import kernels as K
from .layers import _transpose_batched

SLOPE = 0.2  # nn.LeakyReLU(0.2), modules.py:75,78,108,123
RATIOS = (8, 8, 2, 2)  # modules.py:91


def _wn(mod):
    # torch.nn.utils.weight_norm gives the reference's weight_g / weight_v keys (the
    # parametrizations API would rename them); its deprecation warning is noise here
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return nn.utils.weight_norm(mod)


def WNConv1d(*args, **kwargs):
    return _wn(nn.Conv1d(*args, **kwargs))


def WNConvTranspose1d(*args, **kwargs):
    return _wn(nn.ConvTranspose1d(*args, **kwargs))


class ResnetBlock(nn.Module):
    """modules.py:72-86: shortcut(x) + [LeakyReLU, ReflectionPad(d), WNConv(k3, dilation d),
    LeakyReLU, WNConv(k1)](x) -- parameters only (see module docstring)."""

    def __init__(self, dim, dilation=1):
        super().__init__()
        self.dilation = dilation
        self.block = nn.Sequential(
            nn.LeakyReLU(SLOPE),
            nn.ReflectionPad1d(dilation),
            WNConv1d(dim, dim, kernel_size=3, dilation=dilation),
            nn.LeakyReLU(SLOPE),
            WNConv1d(dim, dim, kernel_size=1),
        )
        self.shortcut = WNConv1d(dim, dim, kernel_size=1)


def _pack(conv, stride=0, pad=0):
    """weight_norm + GEMM pack of one (transposed) conv: (W [N][K] in the compute dtype, bias)."""
    v, g = conv.weight_v.detach(), conv.weight_g.detach()
    d0, d1, k = v.shape
    dev = v.device
    tdt = K.compute_torch_dtype()
    if stride:
        w = torch.empty(stride * d1, 3 * d0, device=dev, dtype=tdt)
        bias = torch.empty(stride * d1, device=dev)
    else:
        w = torch.empty(d0, k * d1, device=dev, dtype=tdt)
        bias = None
    norms = torch.empty(d0, device=dev)
    b = conv.bias.detach() if conv.bias is not None else None
    L.call("avc_mg_wn_pack", v.contiguous().data_ptr(), g.contiguous().data_ptr(), K._ptr(b), d0, d1, k, int(stride),
           int(pad), norms.data_ptr(), w.data_ptr(), K._dt(w), K._ptr(bias), K.stream())
    return w, (bias if stride else b)


def _pack_f32(conv):
    """fp32 [taps][C] weight of the output conv (mg_conv_out reads it directly)."""
    v, g = conv.weight_v.detach(), conv.weight_g.detach()
    d0, d1, k = v.shape
    w = torch.empty(d0, k * d1, device=v.device)
    norms = torch.empty(d0, device=v.device)
    L.call("avc_mg_wn_pack", v.contiguous().data_ptr(), g.contiguous().data_ptr(), None, d0, d1, k, 0, 0,
           norms.data_ptr(), w.data_ptr(), K.F32, None, K.stream())
    return w


class Generator(nn.Module):
    """modules.py:88-131 with the reference's constructor and state_dict; forward on HIP."""

    def __init__(self, input_size, ngf, n_residual_layers):
        super().__init__()
        self.hop_length = int(np.prod(RATIOS))
        mult = int(2 ** len(RATIOS))
        model = [nn.ReflectionPad1d(3), WNConv1d(input_size, mult * ngf, kernel_size=7, padding=0)]
        self._stages = []  # (ratio, index of the ConvTranspose1d, [indices of its ResnetBlocks])
        for r in RATIOS:
            model += [nn.LeakyReLU(SLOPE),
                      WNConvTranspose1d(mult * ngf, mult * ngf // 2, kernel_size=r * 2, stride=r,
                                        padding=r // 2 + r % 2, output_padding=r % 2)]
            ct = len(model) - 1
            blocks = []
            for j in range(n_residual_layers):
                model += [ResnetBlock(mult * ngf // 2, dilation=3 ** j)]
                blocks.append(len(model) - 1)
            self._stages.append((r, ct, blocks))
            mult //= 2
        model += [nn.LeakyReLU(SLOPE), nn.ReflectionPad1d(3), WNConv1d(ngf, 1, kernel_size=7, padding=0), nn.Tanh()]
        self._out = len(model) - 2
        self.model = nn.Sequential(*model)
        self.input_size, self.ngf = input_size, ngf
        self._packs = None
        self._pack_key = None

    # ------------------------------------------------------------------ weight packs
    def _key(self):
        return (K.compute(),) + tuple((p.data_ptr(), p._version) for p in self.parameters())

    def packs(self):
        key = self._key()
        if self._packs is None or self._pack_key != key:
            m = self.model
            P = {"in": _pack(m[1])}
            for r, ct, blocks in self._stages:
                P[ct] = _pack(m[ct], stride=r, pad=r // 2 + r % 2)
                for bi in blocks:
                    blk = m[bi]
                    P[bi] = (_pack(blk.block[2]), _pack(blk.block[4]), _pack(blk.shortcut))
            conv = m[self._out]
            P["out"] = (_pack_f32(conv), conv.bias.detach())
            self._packs, self._pack_key = P, key
        return self._packs

    # ------------------------------------------------------------------ forward
    def _gemm(self, M, N, Kd, a, w, bias, out=None, accumulate=False):
        bf = K.compute() == K.BF16
        y = torch.empty(M, N, device=w.device) if out is None else out
        y16 = getattr(y, "_bf16", None) if out is not None else None
        if bf and y16 is None:
            y16 = torch.empty(M, N, device=w.device, dtype=torch.bfloat16)
        K.gemm(M, N, Kd, a, K.operand(w, Kd), y, bias=bias, accumulate=accumulate, c_bf16=y16 if bf else None)
        return K.attach_twin(y, y16) if bf and out is None else y

    def _gather(self, x, B, Lf, C, taps, dil, pad, act):
        src = getattr(x, "_bf16", None)
        src = x if src is None else src
        Lo = Lf + 2 * pad - dil * (taps - 1)
        out = torch.empty(B * Lo, taps * C, device=x.device, dtype=K.compute_torch_dtype())
        L.call("avc_mg_gather", src.data_ptr(), K._dt(src), B, Lf, C, taps, dil, pad, 1, int(act), SLOPE,
               out.data_ptr(), K._dt(out), K.stream())
        return out

    def _act(self, x):
        out = torch.empty(x.shape, device=x.device, dtype=K.compute_torch_dtype())
        bf = out.dtype == torch.bfloat16
        L.call("avc_mg_act", x.data_ptr(), x.numel(), SLOPE, None if bf else out.data_ptr(),
               out.data_ptr() if bf else None, K.stream())
        return out

    @torch.no_grad()
    def frames(self, x, B, T):
        """x: frame-major mel (B*T, input_size) fp32 on the device -> audio (B, T*hop) fp32."""
        K._dev(x)
        if x.dtype != torch.float32 or x.shape != (B * T, self.input_size):
            raise ValueError(f"Generator.frames: expected fp32 ({B * T}, {self.input_size}), got "
                             f"{tuple(x.shape)} {x.dtype}")
        if T <= 3:
            raise ValueError("Generator: ReflectionPad1d(3) needs at least 4 mel frames (modules.py:95)")
        P = self.packs()
        m = self.model
        Lf = T
        C = m[1].weight_v.shape[0]
        w, b = P["in"]
        g = self._gather(x.contiguous(), B, Lf, self.input_size, 7, 1, 3, act=False)
        y = self._gemm(B * Lf, C, 7 * self.input_size, K.operand(g, 7 * self.input_size), w, b)
        for r, ct, blocks in self._stages:
            Cin, Cout = C, m[ct].weight_v.shape[1]
            w, b = P[ct]
            a = self._act(y)  # LeakyReLU before the upsampler (modules.py:99)
            y = self._gemm(B * Lf, r * Cout, 3 * Cin, K.operand(a, Cin, window=(3, 1, Lf, Lf, Cin)), w, b)
            Lf, C = Lf * r, Cout
            y16 = getattr(y, "_bf16", None)  # a view is a new tensor: carry the twin over
            y = K.attach_twin(y.view(B * Lf, C), None if y16 is None else y16.view(B * Lf, C))
            for bi in blocks:
                (w1, b1), (w2, b2), (ws, bs) = P[bi]
                d = m[bi].dilation
                h = self._gather(y, B, Lf, C, 3, d, d, act=True)
                h1 = self._gemm(B * Lf, C, 3 * C, K.operand(h, 3 * C), w1, b1)
                h2 = self._act(h1)
                out = self._gemm(B * Lf, C, C, K.operand(y, C), ws, bs)  # shortcut (modules.py:83-86)
                y = self._gemm(B * Lf, C, C, K.operand(h2, C), w2, b2, out=out, accumulate=True)
        wo, bo = P["out"]
        audio = torch.empty(B * Lf, device=x.device)
        L.call("avc_mg_conv_out", y.data_ptr(), B, Lf, C, 7, wo.data_ptr(), bo.data_ptr(), SLOPE, audio.data_ptr(),
               K.stream())
        return audio.view(B, Lf)

    @torch.no_grad()
    def forward(self, x):
        """x: (B, input_size, T) mel -> (B, 1, T*hop) audio (modules.py:130-131)."""
        B, C, T = x.shape
        xf = _transpose_batched(x.float().contiguous(), B, C, T).view(B * T, C)
        return self.frames(xf, B, T).unsqueeze(1)


class MelVocoder:
    """melgan/interface.py:23-53: `inverse(mel (B, 80, T)) -> (B, T*256)` on the HIP generator.
    The checkpoint is read with torch.load(weights_only=True).  `__call__` (audio -> mel,
    Audio2Mel: librosa's Slaney filterbank + STFT, modules.py:26-69) is not part of the
    conversion path (evaluate.py only calls `inverse`) and is not restated."""

    def __init__(self, device="cuda:0", model_name="multi_speaker", generator=None):
        self.device = torch.device(device)
        if generator is None:
            generator = Generator(80, 32, 3)
            sd = torch.load(f"{model_name}.pt", map_location="cpu", weights_only=True)
            generator.load_state_dict(sd)
        self.mel2wav = generator.to(self.device)

    def __call__(self, audio):
        raise NotImplementedError("MelVocoder.__call__ (Audio2Mel, librosa filterbank) is not on the conversion "
                                  "path and is not restated (autoformer_amd/melgan.py)")

    def inverse(self, mel):
        return self.mel2wav(mel.to(self.device)).squeeze(1)

    def inverse_frames(self, mel_frames):
        """(B, T, 80) frame-major mel (the Converter's output layout) -> (B, T*256): no transpose."""
        B, T, C = mel_frames.shape
        return self.mel2wav.frames(mel_frames.reshape(B * T, C).float().contiguous(), B, T)


def load_model(mel2wav_path, device="cuda:0"):
    """interface.py:12-20 (which ignores its path argument and reads linda_johnson.pt)."""
    g = Generator(80, 32, 3)
    g.load_state_dict(torch.load("linda_johnson.pt", map_location="cpu", weights_only=True))
    return g.to(device)
