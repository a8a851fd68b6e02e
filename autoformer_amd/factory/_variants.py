"""Shared construction of the AdaIN ("2") and speaker-embedding-adjust ("_Adjust") model
variants over the AutoVC / MetaConv / MetaPool families.

AdaIN variants (AutoVC2.py, MetaConv2.py, MetaPool2.py):
  * Encoder gains ``feature_pre_extract`` (3 x ConvNorm(80, 80, linear) + BN, no activation),
    registered FIRST (AutoVC2.py:14-33, MetaConv2.py:86-102); its outputs replace the mel and
    each yields ``[x.mean(), x.std()]`` (AutoVC2.py:56-61).  Encoder.forward returns
    ``(codes, features)``.
  * Postnet gains ``adain`` and ``feature_last_combine`` (3 x ConvNorm(80, 80, linear));
    after the 5 convs: 3 x (AdaIN(x, mu_i, std_i), conv_i) (AutoVC2.py:175-201).
  * forward(x, c_org, c_trg, target_feature=None): (codes, features) when c_trg and
    target_feature are None; otherwise the 3 outputs with the postnet statistics taken from
    target_feature if given, else the source's own (AutoVC2.py:213-242).
Adjust variants (AutoVC_Adjust.py, MetaConv_Adjust.py, MetaPool_Adjust.py):
  * ``adjust = Adjust(dim_emb)`` registered LAST; forward(x, c_org, c_trg, isConvert=False,
    x_target=None) -> (c_org', mel, mel_postnet, codes) with c_org' = adjust(x, c_org)
    (not for MetaPool_Adjust, whose forward leaves c_org as given, MetaPool_Adjust.py:258-260)
    and c_trg' = adjust(x_target if isConvert else x, c_trg) (AutoVC_Adjust.py:177-205).
"""
import torch.nn as nn

from .. import kernels as K
from .. import layers as Lyr
from .. import metaformer as MF
from .. import variants as V
from .Adjust import Adjust
from .AutoVC import Postnet, _conv_bn_block, _frames, decode
from .Norm import AdaIN, ConvNorm


def adain_encoder(Base):
    class Encoder(Base):
        __doc__ = f"{Base.__doc__ or Base.__name__} + feature_pre_extract (AutoVC2.py:14-33, :56-61)."

        def __init__(self, *args, **kw):
            super().__init__(*args, **kw)
            self.feature_pre_extract = nn.ModuleList([_conv_bn_block(80, 80, "linear") for _ in range(3)])
            # registered first in the reference (state_dict / parameter order)
            mods = list(self._modules.items())
            self._modules.clear()
            self._modules.update([mods[-1]] + mods[:-1])
            self._pre = [Lyr.ConvBNCore(s[0].conv, s[1], K.ACT_NONE) for s in self.feature_pre_extract]

        def pre_extract(self, mel, B, T):
            """Frame-major mel -> (features-extracted frames, [[mean, std]] x 3)."""
            h, feats = mel, []
            for core in self._pre:
                h = Lyr.conv_bn(core, h, B, T)
                m = V.moments(h)
                feats.append([m[0], m[1]])
            return h, feats

        def codes_and_features(self, x, c_org):
            mel, B, T = _frames(x)
            h, feats = self.pre_extract(mel, B, T)
            return self.codes_frames(h, c_org, B, T), feats

        def forward(self, x, c_org):
            K.require_device(x, c_org)
            codes, feats = self.codes_and_features(x, c_org)
            return list(codes.split(2 * self.dim_neck, dim=-1)), feats

    Encoder.__name__ = Encoder.__qualname__ = "Encoder"
    return Encoder


class PostnetAdaIN(Postnet):
    """Postnet of the AdaIN variants (AutoVC2.py:123-201)."""

    def __init__(self):
        super().__init__()
        self.adain = AdaIN()
        self.feature_last_combine = nn.ModuleList(
            [nn.Sequential(ConvNorm(80, 80, kernel_size=5, stride=1, padding=2, dilation=1, w_init_gain="linear"))
             for _ in range(3)])
        self._comb = [Lyr.PackCache() for _ in range(3)]

    def frames(self, mel, B, T, features, residual=None):
        h = mel
        for core in self._convs:
            h = Lyr.conv_bn(core, h, B, T)
        for comb, cache, f in zip(self.feature_last_combine, self._comb, features):
            h = V.adain(h, f[0], f[1])
            h = MF.conv(h, comb[0].conv, cache, B, T)
        return h if residual is None else MF.add(residual, h)

    def forward(self, x, features):
        """Reference layout (B, 80, T) in and out."""
        K.require_device(x, features)
        B, C, T = x.shape
        return Lyr.frames_to_bct(self.frames(Lyr.bct_to_frames(x), B, T, features), B, T)


class AdaINModel(nn.Module):
    """forward of AutoVC2 / MetaConv2 / MetaPool2 (AutoVC2.py:213-242)."""

    def forward(self, x, c_org, c_trg, target_feature=None):
        K.require_device(x, c_org, c_trg, target_feature)
        codes, feats = self.encoder.codes_and_features(x, c_org)
        if c_trg is None and target_feature is None:
            return codes, feats
        return decode(self, x, codes, c_trg, target_feature if target_feature is not None else feats)


class AdjustModel(nn.Module):
    """forward of AutoVC_Adjust / MetaConv_Adjust / MetaPool_Adjust (AutoVC_Adjust.py:177-205)."""

    adjusts_org = True

    def add_adjust(self, dim_emb):
        self.adjust = Adjust(dim_emb)

    def forward(self, x, c_org, c_trg, isConvert=False, x_target=None):
        K.require_device(x, c_org, c_trg, x_target)
        # train_with_adjust.py:99 passes emb_org as both c_org and c_trg, so the reference runs
        # Adjust twice on identical inputs (AutoVC_Adjust.py:179, :189): identical outputs, and
        # each BatchNorm's running statistics moved twice.  One pass with two statistics
        # updates gives the same forward, buffers and (summed) gradient at half the cost.
        shared = self.adjusts_org and c_trg is c_org and not isConvert
        if self.adjusts_org:
            c_org = self.adjust(x, c_org, stat_updates=2 if shared else 1)
        codes = self.encoder.codes_flat(x, c_org)
        if c_trg is None:
            return codes
        elif isConvert:
            c_trg = self.adjust(x_target, c_trg)
        elif shared:
            c_trg = c_org
        else:
            # in training c_trg is c_org; in conversion pass the target mel (AutoVC_Adjust.py:186-189)
            c_trg = self.adjust(x, c_trg)
        return (c_org,) + decode(self, x, codes, c_trg)
