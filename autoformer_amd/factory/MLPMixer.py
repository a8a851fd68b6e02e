"""MLP-Mixer parameter container with the reference's module tree and state_dict keys
(/root/reference/factory/MLPMixer.py:16-92): Sequential(Rearrange, Linear,
Sequential(PreNormResidual(LayerNorm, FeedForward(Conv1d k1)), PreNormResidual(LayerNorm,
FeedForward(Linear))), Conv1d(k5)).  The computation is metaformer._MLPMixerFn."""
from functools import partial

import torch.nn as nn

from .. import layers as Lyr


class _Rearrange(nn.Module):
    """Placeholder for einops' Rearrange (no parameters; keeps the Sequential indices)."""

    def __init__(self, patch):
        super().__init__()
        self.patch = patch


def FeedForward(dim, expansion_factor=4, dropout=0.0, dense=nn.Linear):
    return nn.Sequential(dense(dim, dim * expansion_factor), nn.GELU(), nn.Dropout(dropout),
                         dense(dim * expansion_factor, dim), nn.Dropout(dropout))


class PreNormResidual(nn.Module):
    def __init__(self, dim, fn):
        super().__init__()
        self.fn = fn
        self.norm = nn.LayerNorm(dim)


class MLPMixer(nn.Sequential):
    def __init__(self, *, image_size, channels, patch_size, dim, depth, out_dim, kernel_size=5, padding=2,
                 expansion_factor=4, dropout=0.0):
        assert (image_size % patch_size) == 0, "image must be divisible by patch size"
        if depth != 1 or channels != 1 or dropout != 0.0:
            raise NotImplementedError("the MetaFormer path uses depth=1, channels=1, dropout=0")
        num_patches = (image_size // patch_size) ** 2
        chan_first, chan_last = partial(nn.Conv1d, kernel_size=1), nn.Linear
        super().__init__(
            _Rearrange(patch_size),
            nn.Linear((patch_size ** 2) * channels, dim),
            nn.Sequential(PreNormResidual(dim, FeedForward(num_patches, expansion_factor, dropout, chan_first)),
                          PreNormResidual(dim, FeedForward(dim, expansion_factor, dropout, chan_last))),
            nn.Conv1d(num_patches, out_dim, kernel_size=kernel_size, padding=padding),
        )
        self.ps = patch_size
        self.cache = Lyr.PackCache()
        self.tm_cache = Lyr.PackCache()  # token-mixing weights: W1^T and W2 in the compute dtype
        self.cf_cache = Lyr.PackCache()  # patch-embedding / channel-FF weights in the compute dtype

    @property
    def ln_eps(self):
        return (self[2][0].norm.eps, self[2][1].norm.eps)

    def flat_params(self):
        tok, ch = self[2][0], self[2][1]
        return (self[1].weight, self[1].bias, tok.norm.weight, tok.norm.bias, tok.fn[0].weight, tok.fn[0].bias,
                tok.fn[3].weight, tok.fn[3].bias, ch.norm.weight, ch.norm.bias, ch.fn[0].weight, ch.fn[0].bias,
                ch.fn[3].weight, ch.fn[3].bias, self[3].weight, self[3].bias)

    def forward(self, *a, **k):  # pragma: no cover
        raise RuntimeError("MLPMixer is driven by its parent block (metaformer.mlp_mixer)")
