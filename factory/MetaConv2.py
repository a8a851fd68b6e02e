from autoformer_amd.factory.MetaConv2 import *  # noqa: F401,F403
