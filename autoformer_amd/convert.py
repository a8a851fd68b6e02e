"""Voice conversion with a trained plugin model (reference util/evaluate.py:36-94,
Evaluator.crop_mel / get_trans_mel): crop or zero-pad the source (and target) mel to
`len_crop`, run the model with the source and target speaker embeddings -- dispatched like
get_trans_mel over the three model families (plain: model(x, e_org, e_trg); isAdjust:
model(x, e_org, e_trg, True, mel_target), 4 outputs; isAdain: features of the source first,
model(x, e_org, None, None), then model(x, e_org, e_trg, feature)) -- and cut the converted mel
back to the source's real length when it was padded (the `isPlay` branch).

Same kernels as training, forward only under `torch.no_grad()`; the model stays in whatever
BatchNorm mode the caller left it in (the reference converts with the model in train mode, so
BN uses the statistics of the one utterance).  `get_wavs` (evaluate.py:96-98) turns a converted
mel into a waveform with the HIP MelGAN generator (autoformer_amd.melgan.MelVocoder) when the
Converter was given one.
"""
from __future__ import annotations

import numpy as np
import torch


def crop_mel(mel: np.ndarray, len_crop: int, rng=np.random):
    """evaluate.py:36-50: (T, 80) -> ((len_crop, 80), pad_size): zero padding at the end when
    T < len_crop, a uniform crop offset in [0, T - len_crop) when longer (one rng draw)."""
    T = mel.shape[0]
    if T < len_crop:
        out = np.zeros((len_crop,) + mel.shape[1:], dtype=mel.dtype)
        out[:T] = mel
        return out, len_crop - T
    if T == len_crop:
        return mel, 0
    left = rng.randint(0, T - len_crop)
    return mel[left:left + len_crop], 0


class Converter:
    """convert(mel_source, emb_org, emb_trg) -> converted mel (T', 80) on the host."""

    def __init__(self, model, len_crop: int, device="cuda:0", vocoder=None):
        self.model = model
        self.len_crop = len_crop
        self.device = torch.device(device)
        self.vocoder = vocoder  # autoformer_amd.melgan.MelVocoder (evaluate.py:24) or None

    @torch.no_grad()
    def get_wavs(self, mel, frames: bool = False):
        """evaluate.py:96-98: (1, 80, T) mel -> (1, T*256) waveform (the reference contract).
        frames=True: a frame-major (1, T, 80) mel, the layout get_trans_mel returns, goes straight
        in without the transpose.  The layout is stated, never guessed from the shape (T may be 80)."""
        if self.vocoder is None:
            raise RuntimeError("Converter was built without a vocoder (pass vocoder=MelVocoder(...))")
        if mel.dim() != 3 or mel.shape[2 if frames else 1] != 80:
            raise ValueError(f"get_wavs: expected a {'(1, T, 80)' if frames else '(1, 80, T)'} mel, got "
                             f"{tuple(mel.shape)}")
        return self.vocoder.inverse_frames(mel) if frames else self.vocoder.inverse(mel)

    def _dev(self, a):
        return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).unsqueeze(0).to(self.device)

    @torch.no_grad()
    def get_trans_mel(self, mel_source: np.ndarray, mel_target, emb_org: np.ndarray, emb_trg: np.ndarray,
                      isAdjust: bool = False, isAdain: bool = False, isPlay: bool = False):
        """util/evaluate.py:56-94 on host mels: returns (mel_source, mel_target, mel_trans) device
        tensors (1, T, 80) exactly as the reference does; the source is cropped before the target
        (the reference's rng order).  mel_target may be None unless isAdjust."""
        src, pad_s = crop_mel(mel_source, self.len_crop)
        x = self._dev(src)
        y, pad_t = (None, 0)
        if mel_target is not None:
            tgt, pad_t = crop_mel(mel_target, self.len_crop)
            y = self._dev(tgt)
        eo, et = self._dev(emb_org), self._dev(emb_trg)
        if isAdjust:
            if y is None:
                raise ValueError("isAdjust conversion needs the target mel (evaluate.py:79)")
            _, _, mel_trans, _ = self.model(x, eo, et, True, y)
        elif isAdain:
            _, feature = self.model(x, eo, None, None)
            _, mel_trans, _ = self.model(x, eo, et, feature)
        else:
            _, mel_trans, _ = self.model(x, eo, et)
        mel_trans = mel_trans.squeeze(1)
        if isPlay:
            if pad_s > 0:
                x = x[:, : self.len_crop - pad_s, :]
                mel_trans = mel_trans[:, : self.len_crop - pad_s, :]
            if y is not None and pad_t > 0:
                y = y[:, : self.len_crop - pad_t, :]
        return x, y, mel_trans

    @torch.no_grad()
    def convert(self, mel_source: np.ndarray, emb_org: np.ndarray, emb_trg: np.ndarray, trim: bool = True,
                mel_target=None, isAdjust: bool = False, isAdain: bool = False):
        """The converted mel (T', 80) on the host (trimmed to the source length when padded)."""
        _, _, mel_trans = self.get_trans_mel(mel_source, mel_target, emb_org, emb_trg, isAdjust, isAdain,
                                             isPlay=trim)
        return mel_trans[0].float().cpu().numpy()
