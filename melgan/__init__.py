"""Drop-in ``melgan`` package: util/evaluate.py:5 does ``from melgan.interface import *`` and
calls ``MelVocoder(model_name=...).inverse(mel)`` (:24,98).  With this repository first on
PYTHONPATH it gets the HIP generator of autoformer_amd.melgan (reference melgan/)."""
