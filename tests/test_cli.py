"""The C1 driver (python -m autoformer_amd.train, reference train.py:152-168) on the CPU: flags,
Config, the synthetic batches, and the refusal to run the product path anywhere but a GPU."""
import subprocess
import sys

import pytest
import torch

from .conftest import ROOT


def test_parser_has_reference_and_build_flags():
    from autoformer_amd.train import build_parser

    a = build_parser().parse_args(["--model_name", "AutoVC", "--synthetic", "--batch_size", "2", "--len_crop", "128",
                                   "--freq", "16", "--dtype", "bf16", "--num_iters", "5"])
    assert (a.model_name, a.batch_size, a.len_crop, a.freq, a.dtype, int(a.num_iters)) == ("AutoVC", 2, 128, 16,
                                                                                           "bf16", 5)
    d = build_parser().parse_args([])
    # the reference's defaults (train.py:152-159, Config train.py:134-150)
    assert (d.device, int(d.num_iters), d.batch_size, d.len_crop, d.freq, d.log_step) == ("cuda:0", 1000000, 2, 176,
                                                                                          22, 10)


def test_config_mirrors_reference():
    from autoformer_amd.train import Config

    c = Config("AutoVC", None, "cuda:0", 10, False)
    assert (c.lambda_cd, c.dim_neck, c.dim_emb, c.dim_pre, c.freq, c.batch_size, c.len_crop) == (1, 44, 256, 512, 22,
                                                                                                 2, 176)


def test_synthetic_batches_shape_and_determinism():
    from autoformer_amd.train import SyntheticUtterances

    it = iter(SyntheticUtterances(3, 128))
    x0, e0 = next(it)
    x1, _ = next(it)
    assert x0.shape == (3, 128, 80) and e0.shape == (3, 256) and x0.dtype == torch.float32
    assert float(x0.min()) >= -5 and float(x0.max()) <= 2
    assert torch.allclose(e0.norm(dim=1), torch.ones(3), atol=1e-5)
    assert not torch.equal(x0, x1)
    assert torch.equal(next(iter(SyntheticUtterances(3, 128)))[0], x0)


def test_cli_refuses_cpu_device():
    r = subprocess.run([sys.executable, "-m", "autoformer_amd.train", "--synthetic", "--device", "cpu"], cwd=ROOT,
                       capture_output=True, text=True)
    assert r.returncode != 0 and "need a GPU" in r.stderr


def test_cli_needs_data_or_synthetic():
    from autoformer_amd.train import main

    with pytest.raises(SystemExit):
        main(["--model_name", "AutoVC"])
