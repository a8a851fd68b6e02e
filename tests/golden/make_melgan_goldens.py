"""Generate the MelGAN generator fixture from the *reference* module (survey container only).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_melgan_goldens.py

Imports /root/reference/melgan/modules.py (read-only) on the CPU.  That file imports
`librosa.filters.mel` at module level for `Audio2Mel` (modules.py:4,43-45); librosa is not
installed, so a stand-in module whose `mel` raises is placed in sys.modules -- the same
treatment the survey gave `wandb` for train.py.  `Generator` (modules.py:88-131), the code under
test, never calls it.  Weights: autoformer_amd.detinit.det_melgan_state (closed form), loaded
into the reference module; inputs: a closed-form log-mel-like (B=2, 80, T=16) tensor.

Writes melgan_G.npz: mel, audio = Generator(80, 32, 3)(mel) (fp32, no_grad), and the state_dict
key order / shapes.
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)
from autoformer_amd.detinit import det_melgan_state, det_mel  # noqa: E402


def _librosa_mel(*a, **k):
    raise NotImplementedError("librosa is absent; Audio2Mel is not used by Generator")


lib = types.ModuleType("librosa")
filt = types.ModuleType("librosa.filters")
filt.mel = _librosa_mel
lib.filters = filt
sys.modules.setdefault("librosa", lib)
sys.modules.setdefault("librosa.filters", filt)
sys.path.insert(0, "/root/reference")
from melgan.modules import Generator  # noqa: E402

torch.set_num_threads(8)
g = Generator(80, 32, 3)
shapes = [(k, tuple(v.shape)) for k, v in g.state_dict().items()]
sd = det_melgan_state(shapes)
g.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
mel = torch.from_numpy(det_mel(2, 80, 16))
with torch.no_grad():
    audio = g(mel)
np.savez_compressed(os.path.join(HERE, "melgan_G.npz"), mel=mel.numpy(), audio=audio.numpy(),
                    keys=np.array([k for k, _ in shapes]),
                    shapes=np.array([",".join(map(str, s)) for _, s in shapes]))
print("melgan_G.npz", tuple(audio.shape), float(audio.abs().max()), float(audio.std()))
