from autoformer_amd.factory.MetaPool import MetaPool  # noqa: F401
