"""AutoVC_Adjust — AutoVC whose speaker embeddings are refined by Adjust
(/root/reference/factory/AutoVC_Adjust.py).  forward(x, c_org, c_trg, isConvert=False,
x_target=None) -> (c_org', mel, mel_postnet, codes); construction shared in _variants.py."""
from .Adjust import Adjust  # noqa: F401
from .AutoVC import Decoder, Encoder, Postnet
from ._variants import AdjustModel


class AutoVC_Adjust(AdjustModel):
    def __init__(self, dim_neck, dim_emb, dim_pre, freq):
        super().__init__()
        self.encoder = Encoder(dim_neck, dim_emb, freq)
        self.decoder = Decoder(dim_neck, dim_emb, dim_pre)
        self.postnet = Postnet()
        self.add_adjust(dim_emb)
        self.dim_neck = dim_neck
