"""Persistent-recurrence failure is loud (VERDICT r1 'What's weak' 5): a spin timeout inside
lstm_persist_* raises the process fault word, and the training step raises DeviceFault where
the loss is read instead of training on the unfinished outputs."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _trainstep(B=8, T=32):
    import autoformer_amd as A
    from autoformer_amd.detinit import det_init_, det_inputs
    from autoformer_amd.factory.AutoVC import AutoVC
    from autoformer_amd.train import TrainStep

    A.set_compute("bf16")
    m = AutoVC(44, 256, 512, 16)
    det_init_(m)
    m = m.to(DEV).train()
    x, e = det_inputs(B, T, seed=4)
    return TrainStep(m), torch.from_numpy(x).to(DEV), torch.from_numpy(e).to(DEV)


def test_persistent_path_query_matches_occupancy():
    from autoformer_amd import kernels as K

    import autoformer_amd as A
    A.set_compute("bf16")
    # B = 64, H = 1024: 8 groups x 32 members = 256 workgroups, one per CU of the MI355X
    assert K.lstm_persistent_fwd(64, 1024, 1) and K.lstm_persistent_bwd(64, 1024, 1)
    assert K.lstm_persistent_fwd(64, 512, 1) and K.lstm_persistent_bwd(64, 512, 1)
    # 9 groups x 32 = 288 workgroups cannot all be resident: per-step kernels instead
    assert not K.lstm_persistent_fwd(72, 1024, 1) and not K.lstm_persistent_bwd(72, 1024, 1)
    assert not K.lstm_persistent_fwd(64, 1024, 2)  # bidirectional: per-step path
    A.set_compute("fp32")
    assert not K.lstm_persistent_fwd(64, 1024, 1)
    A.set_compute("bf16")


def test_forced_spin_timeout_raises_at_loss_read():
    from autoformer_amd import kernels as K
    from autoformer_amd.layers import set_grad_sink

    ts, x, e = _trainstep()
    try:
        K.clear_faults()
        ts.step(x, e)
        ts.check()  # healthy step: no fault
        K.lstm_set_spin(-1)  # injected: every wait of the persistent recurrences times out
        ts.step(x, e)
        with pytest.raises(K.DeviceFault, match="spin timeout"):
            ts.check()
        # the asynchronous probe raises at the next step as well
        K.lstm_set_spin(0)
        torch.cuda.synchronize()
        with pytest.raises(K.DeviceFault):
            ts.step(x, e)
    finally:
        K.lstm_set_spin(0)
        torch.cuda.synchronize()
        K.clear_faults()
        set_grad_sink(False)


def test_solver_raises_on_fault():
    """Solver reads the losses with .item() every step (train.py:103-105): it checks the
    fault word there."""
    import autoformer_amd as A
    from autoformer_amd import kernels as K
    from autoformer_amd.detinit import det_inputs
    from autoformer_amd.train import Solver

    A.set_compute("bf16")
    x, e = det_inputs(8, 32, seed=6)

    class Cfg:
        lambda_cd, dim_neck, dim_emb, dim_pre, freq = 1, 44, 256, 512, 16
        model_name, batch_size, num_iters, device, log_step = "AutoVC", 8, 2, DEV, 10

    s = Solver([(torch.from_numpy(x), torch.from_numpy(e))], Cfg())
    try:
        K.clear_faults()
        K.lstm_set_spin(-1)
        with pytest.raises(K.DeviceFault):
            s.train()
    finally:
        K.lstm_set_spin(0)
        torch.cuda.synchronize()
        K.clear_faults()
