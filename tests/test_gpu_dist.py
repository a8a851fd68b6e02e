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
        from autoformer_amd import kernels as K

        # the collective / recurrence ordering invariant was checked at every decoder
        # recurrence launch of the eager and the recorded steps, with collectives in flight
        st = K.ordering_stats()
        assert st["checks"] > 0 and not K.collectives_outstanding()
        if ts.world > 1 and overlapped:
            assert st["enqueued"] > 0
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
# Two ranks, one GPU each, over RCCL in bf16: the persistent recurrences run beside the collectives.
# Sharing ONE GPU between two bf16 ranks is never done: two processes' whole-chip persistent grids
# can interleave their workgroups and wait on each other (hence fp32 in the gloo tests above).
# Cases (each rank sees the same batches, so the average equals the single-process gradient):
#   small  B=16 T=64, eager, 2 steps, default split-K (atomics: close, not bit-equal, to one process)
#   bench  the bench.py C2 path: B=64 T=128 freq=16, 1 eager step, the recorded step, 5 replays, each
#          step a new batch; deterministic mode (no split-K atomics), so one process stepping eagerly
#          on the same batches must be matched to the bit (the average of two identical gradients is
#          exact, and a replay is bit-identical to the eager step: tests/test_gpu_replay.py)
#   c5     the same for BASELINE C5 (train_with_discriminator.py:90-111): AutoVC + Discriminator,
#          T=176 freq=22, one flat buffer / one Adam over both models (bench.py --disc)
_CASES = {"small": dict(B=16, T=64, freq=FREQ, steps=2, record=False, det=False, disc=False),
          "bench": dict(B=64, T=128, freq=16, steps=7, record=True, det=True, disc=False),
          "c5": dict(B=64, T=176, freq=22, steps=7, record=True, det=True, disc=True)}


def _nccl_worker(rank, world, port, q, case):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import torch.distributed as dist

    try:
        torch.cuda.set_device(rank)
        from autoformer_amd import dist as D

        D.init_from_env("nccl")
        assert dist.get_backend() == "nccl"
        q.put((rank,) + _run_bf16(f"cuda:{rank}", case))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as exc:
        q.put((rank, repr(exc), None, None))
        raise


def _run_bf16(dev, case, replay=None):
    """One rank (or the single-process reference, replay=False) of a case: (flat params after the
    last step, the losses of every step, whether the persistent recurrences ran)."""
    import autoformer_amd as A
    from autoformer_amd import kernels as K
    from autoformer_amd.detinit import det_init_, det_inputs
    from autoformer_amd.factory.AutoVC import AutoVC
    from autoformer_amd.layers import set_grad_sink
    from autoformer_amd.train import TrainStep, gan_extra

    c = _CASES[case]
    B, T = c["B"], c["T"]
    replay = c["record"] if replay is None else replay
    A.set_compute("bf16")
    K.set_deterministic(c["det"])
    m = AutoVC(44, 256, 512, c["freq"])
    det_init_(m)
    m = m.to(dev).train()
    if c["disc"]:
        from autoformer_amd.factory.Discriminator import Discriminator

        disc = Discriminator(crop_len=T)
        det_init_(disc)
        disc = disc.to(dev).train()
        ts = TrainStep(m, lr=1e-4, extra=gan_extra(disc), extra_modules=[disc])
    else:
        ts = TrainStep(m, lr=1e-4)
    batches = [tuple(torch.from_numpy(a).to(dev) for a in det_inputs(B, T, seed=40 + i)) for i in range(c["steps"])]
    losses = []
    try:
        if c["record"]:
            xb, eb = batches[1][0].clone(), batches[1][1].clone()
        for i, (x, e) in enumerate(batches):
            if replay and i == 1:
                ts.record(xb, eb, warmup=0)
                loss = ts.loss
            else:
                loss = ts.step(x, e)  # a replay copies the batch into the recorded input tensors
            losses.append(float(loss.item()))
        ts.check()
        assert not K.collectives_outstanding()
    finally:
        set_grad_sink(False)
        K.set_deterministic(False)
    return ts.flat.cpu().numpy(), losses, K.lstm2_bwd_persistent(B, 1024)


def _run_world2_nccl(case):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_nccl_worker, args=(r, 2, port, q, case)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        rank, flat, losses, pers = q.get(timeout=400)
        assert not isinstance(flat, str), flat
        assert pers, "the persistent recurrences did not run"
        res[rank] = (torch.from_numpy(flat), losses)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return res


@pytest.mark.timeout(300)
@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="RCCL needs one GPU per rank (>= 2 GPUs)")
def test_dp_world2_nccl_bf16_persistent():
    """Two ranks over RCCL, bf16 with the persistent recurrences (the production kernels), the
    decoder-slice all-reduce overlapped with the encoder backward: both ranks end bit-identical,
    and close to one process stepping the same batch (the ranks see identical batches, so the
    average equals the single-process gradient up to split-K atomic ordering)."""
    single, _, persistent = _run_bf16("cuda:0", "small")
    assert persistent
    res = _run_world2_nccl("small")
    (r0, _), (r1, _) = res[0], res[1]
    single = torch.from_numpy(single)
    torch.testing.assert_close(r0, r1, rtol=0, atol=0)
    # Adam normalises the (analytically zero) gradients of BN-fed conv biases, so those may move
    # by up to ~2 lr under reordered atomics: absolute tolerance 3e-4
    torch.testing.assert_close(r0, single, rtol=1e-3, atol=3e-4)


@pytest.mark.timeout(400)
@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="RCCL needs one GPU per rank (>= 2 GPUs)")
@pytest.mark.parametrize("case", ["bench", "c5"])
def test_dp_world2_nccl_recorded_replay_matches_eager(case):
    """the data-parallel path bench.py --gpus N times (C3: the recorded replay at
    B=64 T=128 with replay.collective re-issuing both RCCL all-reduces; C5: the two-model step) on
    two GPUs, 1 eager + 1 recorded + 5 replayed steps on new batches, against one process stepping
    eagerly on the same batches: identical losses and parameters (deterministic mode)."""
    single, single_losses, persistent = _run_bf16("cuda:0", case, replay=False)
    assert persistent
    res = _run_world2_nccl(case)
    (r0, l0), (r1, l1) = res[0], res[1]
    single = torch.from_numpy(single)
    torch.testing.assert_close(r0, r1, rtol=0, atol=0)
    assert l0 == l1
    torch.testing.assert_close(r0, single, rtol=1e-6, atol=1e-8)
    np_l0, np_single = torch.tensor(l0), torch.tensor(single_losses)
    torch.testing.assert_close(np_l0, np_single, rtol=1e-6, atol=0)
