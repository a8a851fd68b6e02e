"""The C1 driver on the GPU (python -m autoformer_amd.train --synthetic, reference train.py:152-195)
against its CPU counterpart, the oracle Solver (oracle/autovc_cpu.py OracleSolver, train.py:13-132
restated), on the same synthetic batches and closed-form weights: the logged losses of 3 Adam
iterations in fp32 compute, at the bar of the golden 3-step test (rtol 2e-3)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_cli_three_iterations_match_oracle_solver():
    from autoformer_amd.detinit import det_inputs
    from autoformer_amd.train import main
    from oracle import autovc_cpu as O

    B, T, freq = 2, 128, 16
    got = main(["--model_name", "AutoVC", "--synthetic", "--det_init", "--num_iters", "3", "--batch_size", str(B),
                "--len_crop", str(T), "--freq", str(freq), "--dtype", "fp32", "--log_step", "1"])
    s = O.OracleSolver(freq=freq)
    ref = []
    for i in range(3):
        x, e = det_inputs(B, T, seed=1234 + i)
        ref.append(s.step(torch.from_numpy(x), torch.from_numpy(e)))
    np.testing.assert_allclose(np.array(got), np.array(ref), rtol=2e-3)


def test_cli_bf16_discriminator_step_runs():
    from autoformer_amd.train import main

    got = main(["--model_name", "AutoVC", "--synthetic", "--discriminator", "--num_iters", "2", "--batch_size", "4",
                "--len_crop", "176", "--freq", "22", "--dtype", "bf16", "--log_step", "1"])
    assert np.isfinite(np.array(got)).all() and len(got) == 2 and len(got[0]) == 4
