"""Voice conversion with a trained plugin model (reference util/evaluate.py:36-94,
Evaluator.crop_mel / get_trans_mel, AutoVC path): crop or zero-pad the source mel to
`len_crop`, run the model with the source and target speaker embeddings, and cut the
converted mel back to the source's real length when it was padded (the `isPlay` branch).

Same kernels as training, forward only under `torch.no_grad()`; the model stays in whatever
BatchNorm mode the caller left it in (the reference converts with the model in train mode, so
BN uses the statistics of the one utterance).  The MelGAN vocoder that turns the mel into a
waveform is out of scope.
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

    def __init__(self, model, len_crop: int, device="cuda:0"):
        self.model = model
        self.len_crop = len_crop
        self.device = torch.device(device)

    @torch.no_grad()
    def convert(self, mel_source: np.ndarray, emb_org: np.ndarray, emb_trg: np.ndarray, trim: bool = True):
        mel, pad = crop_mel(mel_source, self.len_crop)
        x = torch.from_numpy(np.ascontiguousarray(mel, dtype=np.float32)).unsqueeze(0).to(self.device)
        eo = torch.from_numpy(np.asarray(emb_org, dtype=np.float32)).unsqueeze(0).to(self.device)
        et = torch.from_numpy(np.asarray(emb_trg, dtype=np.float32)).unsqueeze(0).to(self.device)
        _, mel_trans, _ = self.model(x, eo, et)
        out = mel_trans.squeeze(1)[0]
        if trim and pad > 0:
            out = out[: self.len_crop - pad]
        return out.float().cpu().numpy()
