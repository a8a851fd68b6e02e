from autoformer_amd.factory.AutoVC_Adjust import *  # noqa: F401,F403
