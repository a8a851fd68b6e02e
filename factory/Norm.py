from autoformer_amd.factory.Norm import ConvNorm, GroupNorm, LinearNorm, PatchEmbed  # noqa: F401
