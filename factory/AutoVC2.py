from autoformer_amd.factory.AutoVC2 import *  # noqa: F401,F403
