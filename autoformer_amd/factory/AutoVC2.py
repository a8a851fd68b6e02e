"""AutoVC2 — AutoVC with AdaIN feature statistics (/root/reference/factory/AutoVC2.py).
Same constructor and forward(x, c_org, c_trg, target_feature=None) contract, same
state_dict keys; construction shared in _variants.py."""
from . import AutoVC as _base
from ._variants import AdaINModel, PostnetAdaIN, adain_encoder

Encoder = adain_encoder(_base.Encoder)
Decoder = _base.Decoder
Postnet = PostnetAdaIN


class AutoVC2(AdaINModel):
    def __init__(self, dim_neck, dim_emb, dim_pre, freq):
        super().__init__()
        self.encoder = Encoder(dim_neck, dim_emb, freq)
        self.decoder = Decoder(dim_neck, dim_emb, dim_pre)
        self.postnet = Postnet()
        self.dim_neck = dim_neck
