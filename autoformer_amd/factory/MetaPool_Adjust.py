"""MetaPool_Adjust (/root/reference/factory/MetaPool_Adjust.py; class ``MetaPool``)."""
from .MetaConv_Adjust import Adjust, Decoder, Encoder, MetaPool, MetaPool_Adjust, Postnet  # noqa: F401
