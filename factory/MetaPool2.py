from autoformer_amd.factory.MetaPool2 import *  # noqa: F401,F403
