from autoformer_amd.factory.MetaPool_Adjust import *  # noqa: F401,F403
