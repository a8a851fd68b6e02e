"""Data-parallel TrainStep on the MI355X with two ranks sharing one GPU (gloo backend, fp32
compute so the per-step LSTM kernels run instead of the whole-GPU persistent ones): with
identical batches on both ranks the overlapped gradient average (decoder/postnet slice during
the encoder backward, encoder slice after it) must leave the parameters exactly where a
single-process step puts them."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

B, T, FREQ = 2, 32, 16


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_steps(name="AutoVC", steps=2, replay=False):
    import importlib

    import autoformer_amd as A
    from autoformer_amd.detinit import det_init_, det_inputs
    from autoformer_amd.layers import set_grad_sink
    from autoformer_amd.train import TrainStep

    A.set_compute("fp32")
    m = getattr(importlib.import_module(f"autoformer_amd.factory.{name}"), name)(44, 256, 512, FREQ)
    det_init_(m)
    m = m.to("cuda:0").train()
    x, e = det_inputs(B, T, seed=11)
    x, e = torch.from_numpy(x).cuda(), torch.from_numpy(e).cuda()
    ts = TrainStep(m, lr=1e-4)
    try:
        for i in range(steps):
            if replay and i == 1:
                ts.record(x, e, warmup=0)  # the recorded step is step 1; later steps replay it
            else:
                ts.step(x, e)
        torch.cuda.synchronize()
        overlapped = ts.split is not None
    finally:
        set_grad_sink(False)
    return ts.flat.cpu().numpy(), overlapped  # numpy: pickled by value through the queue


def _worker(rank, world, port, q, name, steps=2, replay=False):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import torch.distributed as dist

    from autoformer_amd import dist as D

    try:
        D.init_from_env("gloo")
        flat, overlapped = _run_steps(name, steps, replay)
        q.put((rank, flat, overlapped))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as exc:  # surface worker failures to the parent
        q.put((rank, repr(exc), None))
        raise


# AutoVC and the AdaIN variant overlap the decoder-slice all-reduce with the encoder backward;
# the Adjust variant's `adjust` gradients complete only with the encoder's, so it averages
# everything after the backward (TrainStep.split is None)
@pytest.mark.timeout(240)
@pytest.mark.parametrize("name,expect_overlap", [("AutoVC", True), ("AutoVC2", True), ("AutoVC_Adjust", False)])
def test_dp_world2_overlapped_allreduce_matches_single_process(name, expect_overlap):
    single, _ = _run_steps(name)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, name)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        rank, flat, overlapped = q.get(timeout=200)
        assert not isinstance(flat, str), flat
        assert overlapped == expect_overlap, "unexpected all-reduce overlap mode"
        res[rank] = flat
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    r0, r1, single = (torch.from_numpy(a) for a in (res[0], res[1], single))
    torch.testing.assert_close(r0, r1, rtol=0, atol=0)
    torch.testing.assert_close(r0, single, rtol=1e-5, atol=1e-7)


@pytest.mark.timeout(240)
@pytest.mark.parametrize("name,expect_overlap", [("AutoVC", True), ("AutoVC_Adjust", False)])
def test_dp_world2_recorded_replay_matches_single_process(name, expect_overlap):
    """The recorded step with world 2 (TrainStep.record): the gradient averages are re-issued at
    their places on the comm / main streams by replay.collective at every replay; 4 steps (eager,
    recorded, 2 replays) must land where 4 eager single-process steps do."""
    single, _ = _run_steps(name, steps=4)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, name, 4, True)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        rank, flat, overlapped = q.get(timeout=200)
        assert not isinstance(flat, str), flat
        assert overlapped == expect_overlap
        res[rank] = flat
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    r0, r1, single = (torch.from_numpy(a) for a in (res[0], res[1], single))
    torch.testing.assert_close(r0, r1, rtol=0, atol=0)
    torch.testing.assert_close(r0, single, rtol=1e-5, atol=1e-7)


# ---------------------------------------------------------------------------- RCCL (nccl backend)
def _nccl_worker(rank, world, port, q, B, T):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import torch.distributed as dist

    try:
        torch.cuda.set_device(rank)
        from autoformer_amd import dist as D

        D.init_from_env("nccl")
        assert dist.get_backend() == "nccl"
        flat, persistent = _run_bf16(f"cuda:{rank}", B, T)
        q.put((rank, flat, persistent))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as exc:
        q.put((rank, repr(exc), None))
        raise


def _run_bf16(dev, B, T, steps=2):
    import autoformer_amd as A
    from autoformer_amd import kernels as K
    from autoformer_amd.detinit import det_init_, det_inputs
    from autoformer_amd.factory.AutoVC import AutoVC
    from autoformer_amd.layers import set_grad_sink
    from autoformer_amd.train import TrainStep

    A.set_compute("bf16")
    m = AutoVC(44, 256, 512, FREQ)
    det_init_(m)
    m = m.to(dev).train()
    x, e = det_inputs(B, T, seed=11)
    x, e = torch.from_numpy(x).to(dev), torch.from_numpy(e).to(dev)
    ts = TrainStep(m, lr=1e-4)
    try:
        for _ in range(steps):
            ts.step(x, e)
        ts.check()
    finally:
        set_grad_sink(False)
    return ts.flat.cpu().numpy(), K.lstm_persistent_bwd(B, 1024, 1)


@pytest.mark.timeout(300)
@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="RCCL needs one GPU per rank (>= 2 GPUs)")
def test_dp_world2_nccl_bf16_persistent():
    """Two ranks over RCCL, bf16 with the persistent recurrences (the production kernels), the
    decoder-slice all-reduce overlapped with the encoder backward: both ranks end bit-identical,
    and close to one process stepping the same batch (the ranks see identical batches, so the
    average equals the single-process gradient up to split-K atomic ordering)."""
    B, T = 16, 64
    single, persistent = _run_bf16("cuda:0", B, T)
    assert persistent
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_nccl_worker, args=(r, 2, port, q, B, T)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        rank, flat, pers = q.get(timeout=240)
        assert not isinstance(flat, str), flat
        assert pers
        res[rank] = flat
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    r0, r1, single = (torch.from_numpy(a) for a in (res[0], res[1], single))
    torch.testing.assert_close(r0, r1, rtol=0, atol=0)
    # Adam normalises the (analytically zero) gradients of BN-fed conv biases, so those may move
    # by up to ~2 lr under reordered atomics: absolute tolerance 3e-4
    torch.testing.assert_close(r0, single, rtol=1e-3, atol=3e-4)
