"""MetaConv_Adjust / MetaPool_Adjust (/root/reference/factory/MetaConv_Adjust.py,
MetaPool_Adjust.py): MetaConv / MetaPool with Adjust-refined speaker embeddings."""
from .Adjust import Adjust  # noqa: F401
from .AutoVC import Postnet
from .MetaConv import Decoder, Encoder, MetaBlock  # noqa: F401
from ._variants import AdjustModel


class MetaConv_Adjust(AdjustModel):
    _pool = False

    def __init__(self, dim_neck, dim_emb, dim_pre, freq):
        super().__init__()
        self.encoder = Encoder(dim_neck, freq, dim_pre, pool=self._pool)
        self.decoder = Decoder(dim_pre, pool=self._pool)
        self.postnet = Postnet()
        self.add_adjust(dim_emb)
        self.dim_neck = dim_neck


class MetaPool(MetaConv_Adjust):
    """MetaPool_Adjust.py:250 names this class ``MetaPool``; its forward never adjusts c_org
    (MetaPool_Adjust.py:258-260) and returns it as given."""

    _pool = True
    adjusts_org = False


# the reference module has no ``MetaPool_Adjust`` attribute, so train_with_adjust.py's
# getattr(module, model_name) lookup fails for it there; the alias makes the lookup work
MetaPool_Adjust = MetaPool
