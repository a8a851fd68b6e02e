"""MetaConv (and, with pool=True, MetaPool) on MI355X — drop-in for
/root/reference/factory/MetaConv.py and factory/MetaPool.py (same constructors
``(dim_neck, dim, dim_pre, freq)``, same forward contract and state_dict keys).

Layouts are frame-major (B*L, C).  The encoder runs over time (T must equal crop_len =
176: MetaConv.py:13,92,98 hard-wire it); the decoder treats TIME AS CHANNELS and runs its
convs over the 344-wide code+embedding axis (MetaConv.py:138-179), so its input and the
MLP output are transposed once each, explicitly.
"""
import torch.nn as nn

from .. import kernels as K
from .. import layers as Lyr
from .. import metaformer as MF
from .AutoVC import Postnet, _frames, decode
from .MLPMixer import MLPMixer
from .Norm import ConvNorm, GroupNorm, LinearNorm, PatchEmbed


def _conv_bn_relu(cin, cout, gain="relu"):
    return nn.Sequential(ConvNorm(cin, cout, kernel_size=5, padding=2, w_init_gain=gain), nn.BatchNorm1d(cout),
                         nn.ReLU())


class Pooling(nn.Module):
    """AvgPool1d(pool_size, 1, pool_size//2, count_include_pad=False)(x) - x (MetaPool.py:7-15)."""

    def __init__(self, pool_size=3):
        super().__init__()
        if pool_size != 3:
            raise NotImplementedError("pool_size 3 only (MetaPool.py:20)")


class MetaBlock(nn.Module):
    def __init__(self, dim, source_emb=512, crop_len=176, out_dim_neck=88, patch_size=8, mlp_depth=1, pool=False):
        super().__init__()
        self.norm1 = GroupNorm(dim)
        self.pool = pool
        if pool:
            self.token_mixer = Pooling(3)
        else:
            self.token_mixer = _conv_bn_relu(source_emb, source_emb)
        self.norm2 = GroupNorm(crop_len)
        self.conv_1 = _conv_bn_relu(source_emb, crop_len)
        self.mlp = MLPMixer(image_size=crop_len, channels=1, patch_size=patch_size, dim=crop_len, depth=mlp_depth,
                            out_dim=out_dim_neck)
        self.conv_2 = _conv_bn_relu(out_dim_neck, source_emb)
        self.crop_len = crop_len
        if not pool:
            self._mix = Lyr.ConvBNCore(self.token_mixer[0].conv, self.token_mixer[1], K.ACT_RELU)
        self._c1 = Lyr.ConvBNCore(self.conv_1[0].conv, self.conv_1[1], K.ACT_RELU)
        self._c2 = Lyr.ConvBNCore(self.conv_2[0].conv, self.conv_2[1], K.ACT_RELU)

    def frames(self, x, B, L):
        """MetaConv.py:64-76 on frame-major x (B*L, 512); L must equal crop_len."""
        if L != self.crop_len:
            raise RuntimeError(f"MetaBlock needs L == crop_len ({self.crop_len}), got {L}")
        y = MF.group_norm(x, B, self.norm1, twin=not self.pool)  # the conv mixer reads it as a bf16 operand
        # the residual adds ride on the BN-apply pass of the conv branch (x + relu(bn(conv(.))))
        x = MF.add(x, MF.pool_mixer(y, B, L)) if self.pool else Lyr.conv_bn(self._mix, y, B, L, residual=x)
        a = Lyr.conv_bn(self._c1, x, B, L)
        m = MF.mlp_mixer(MF.group_norm(a, B, self.norm2), self.mlp, B, L)
        return Lyr.conv_bn(self._c2, m, B, L, residual=x)


class Encoder(nn.Module):
    def __init__(self, dim_neck, freq, dim, num_layers=3, pool=False):
        super().__init__()
        self.freq = freq
        self.dim_neck = dim_neck
        self.embding = PatchEmbed()
        self.metablock = nn.Sequential(*[MetaBlock(dim, pool=pool) for _ in range(num_layers)])
        self.output_conv = _conv_bn_relu(512, 176)
        self.mlp = MLPMixer(image_size=176, channels=1, patch_size=16, dim=176, depth=1, out_dim=2 * dim_neck)
        self._emb = Lyr.PackCache()
        self._out = Lyr.ConvBNCore(self.output_conv[0].conv, self.output_conv[1], K.ACT_RELU)

    def codes_flat(self, x, c_org):
        mel, B, T = _frames(x)
        return self.codes_frames(mel, c_org, B, T)

    def codes_frames(self, mel, c_org, B, T):
        if T % self.freq:
            raise IndexError(f"len_crop {T} is not a multiple of freq {self.freq}")
        h = MF.enc_embed(mel, c_org.contiguous(), self.embding.proj, self._emb, B, T)
        for blk in self.metablock:
            h = blk.frames(h, B, T)
        h = Lyr.conv_bn(self._out, h, B, T)
        h = MF.mlp_mixer(h, self.mlp, B, T)  # (B*176, 2*dim_neck) == outputs (B, T, 2*dim_neck)
        return Lyr.codes(h, B, T, self.dim_neck, self.freq)

    def forward(self, x, c_org):
        K.require_device(x, c_org)
        return list(self.codes_flat(x, c_org).split(2 * self.dim_neck, dim=-1))


class Decoder(nn.Module):
    def __init__(self, dim, num_layers=1, pool=False):
        super().__init__()
        self.embding = PatchEmbed(in_chans=176)
        self.metablock = nn.Sequential(
            *[MetaBlock(dim, crop_len=344, patch_size=8, out_dim_neck=88, pool=pool) for _ in range(num_layers)])
        self.output_conv_1 = _conv_bn_relu(512, 344)
        self.mlp = MLPMixer(image_size=344, channels=1, patch_size=8, dim=344, depth=1, out_dim=88)
        self.output_conv_2 = _conv_bn_relu(344, 176)
        self.linear_projection = LinearNorm(88, 80)
        self._emb = Lyr.PackCache()
        self._o1 = Lyr.ConvBNCore(self.output_conv_1[0].conv, self.output_conv_1[1], K.ACT_RELU)
        self._o2 = Lyr.ConvBNCore(self.output_conv_2[0].conv, self.output_conv_2[1], K.ACT_RELU)
        self._lin = Lyr.PackCache()

    def frames(self, enc_out, B, T):
        """enc_out (B*T, 344) = reference (B, C=T, L=344) -> mel (B*T, 80)."""
        W = enc_out.shape[1]
        x = MF.transpose(enc_out, B, T, W)                    # (B*344, T): 344 positions x T channels
        h = MF.conv(x, self.embding.proj, self._emb, B, W)     # (B*344, 512)
        for blk in self.metablock:
            h = blk.frames(h, B, W)
        h = Lyr.conv_bn(self._o1, h, B, W)                     # (B*344, 344)
        m = MF.mlp_mixer(h, self.mlp, B, W)                    # (B*344, 88) == reference (B, 88, 344)
        m = MF.transpose(m, B, W, 88)                          # (B*88, 344): 88 positions x 344 channels
        h2 = Lyr.conv_bn(self._o2, m, B, 88)                   # (B*88, T)
        h2 = MF.transpose(h2, B, 88, T)                        # (B*T, 88)
        lin = self.linear_projection.linear_layer
        return Lyr.linear(h2, lin.weight, lin.bias, self._lin)

    def forward(self, x):
        K.require_device(x)
        xf, B, T = _frames(x)
        return self.frames(xf, B, T).view(B, T, -1)


class MetaConv(nn.Module):
    _pool = False

    def __init__(self, dim_neck, dim, dim_pre, freq):
        super().__init__()
        self.encoder = Encoder(dim_neck, freq, dim_pre, pool=self._pool)
        self.decoder = Decoder(dim_pre, pool=self._pool)
        self.postnet = Postnet()
        self.dim_neck = dim_neck

    def forward(self, x, c_org, c_trg):
        K.require_device(x, c_org, c_trg)
        codes = self.encoder.codes_flat(x, c_org)
        if c_trg is None:
            return codes
        return decode(self, x, codes, c_trg)
