from autoformer_amd.factory.Discriminator import Discriminator  # noqa: F401
