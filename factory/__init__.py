"""Drop-in ``factory`` package: the reference trainers import ``factory.<Model>`` by name
(train.py:45-47, train_with_discriminator.py:43-45,7).  Put this repository first on
PYTHONPATH and they get the MI355X implementations from autoformer_amd.factory."""
