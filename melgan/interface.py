from autoformer_amd.melgan import Generator, MelVocoder, load_model  # noqa: F401
