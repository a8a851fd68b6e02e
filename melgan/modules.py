from autoformer_amd.melgan import Generator, ResnetBlock, WNConv1d, WNConvTranspose1d  # noqa: F401
