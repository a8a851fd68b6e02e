"""MetaConv2 / MetaPool2 — MetaConv / MetaPool with AdaIN feature statistics
(/root/reference/factory/MetaConv2.py, MetaPool2.py); construction shared in _variants.py."""
from . import MetaConv as _base
from ._variants import AdaINModel, PostnetAdaIN, adain_encoder

MetaBlock = _base.MetaBlock
Encoder = adain_encoder(_base.Encoder)
Decoder = _base.Decoder
Postnet = PostnetAdaIN


class MetaConv2(AdaINModel):
    _pool = False

    def __init__(self, dim_neck, dim, dim_pre, freq):
        super().__init__()
        self.encoder = Encoder(dim_neck, freq, dim_pre, pool=self._pool)
        self.decoder = Decoder(dim_pre, pool=self._pool)
        self.postnet = Postnet()
        self.dim_neck = dim_neck


class MetaPool2(MetaConv2):
    _pool = True
