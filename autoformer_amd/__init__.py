"""autoformer_amd — MI355X-native (gfx950) AutoVC / MetaConv / MetaPool training path.

Drop-in for achyun/Autoformer's ``factory`` plugin modules; compute runs in hand-written
HIP kernels (libautovc_hip.so) bound through a C-ABI.  See DESIGN.md.
"""
from .kernels import compute, set_compute  # noqa: F401
from .layers import weights_changed  # noqa: F401

__version__ = "0.1.0"
