from autoformer_amd.factory.MLPMixer import *  # noqa: F401,F403
