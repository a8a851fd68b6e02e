from autoformer_amd.factory.Adjust import *  # noqa: F401,F403
