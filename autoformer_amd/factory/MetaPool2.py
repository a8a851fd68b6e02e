"""MetaPool2 (/root/reference/factory/MetaPool2.py): MetaConv2 with the pooling token mixer."""
from .MetaConv2 import Decoder, Encoder, MetaPool2, Postnet  # noqa: F401
