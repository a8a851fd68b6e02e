from autoformer_amd.factory.MetaConv import MetaBlock, Encoder, Decoder, Postnet, MetaConv  # noqa: F401
