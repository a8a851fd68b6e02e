from autoformer_amd.factory.Norm import ConvNorm, GroupNorm, LinearNorm, PatchEmbed, AdaIN, IN  # noqa: F401
