from autoformer_amd.factory.AutoVC import AutoVC, Decoder, Encoder, Postnet  # noqa: F401
