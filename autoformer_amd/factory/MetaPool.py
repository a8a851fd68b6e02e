"""MetaPool — MetaConv with the Pooling token mixer (/root/reference/factory/MetaPool.py)."""
from .MetaConv import MetaConv


class MetaPool(MetaConv):
    _pool = True
