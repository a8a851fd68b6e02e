from autoformer_amd.factory.MetaConv_Adjust import *  # noqa: F401,F403
