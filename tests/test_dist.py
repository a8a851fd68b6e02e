"""Data-parallel plumbing (dist.py) with world_size 2 on gloo, CPU only: rendezvous from the
torchrun-style environment, parameter flattening, rank-0 broadcast, bucketed gradient mean."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import torch.distributed as dist

    from autoformer_amd import dist as D

    try:
        r, w, local = D.init_from_env("gloo")
        assert (r, w, local) == (rank, world, rank)
        torch.manual_seed(100 + rank)  # ranks start from different weights
        m = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.Conv1d(5, 3, 3))
        params, flat, gflat = D.flatten_params_(m, device=torch.device("cpu"))
        assert flat.numel() == D.param_offsets(params)[1] >= sum(p.numel() for p in m.parameters())
        assert all(p.data_ptr() >= flat.data_ptr() for p in params)
        assert all((p.data_ptr() - flat.data_ptr()) % (4 * D.PARAM_ALIGN) == 0 for p in params)
        D.broadcast_(flat)
        # gradients: rank-dependent, averaged in 3 small buckets (bucket_bytes=64 -> 16 floats)
        gflat.copy_(torch.arange(gflat.numel(), dtype=torch.float32) * (rank + 1))
        D.allreduce_mean_(gflat, bucket_bytes=64)
        # overlapped form: the late slice [split:] first, then the head, as TrainStep does
        split = D.split_offset(params, params[2])  # the conv weight starts the "decoder" part
        assert split == D.param_offsets(params)[0][2]
        g2 = torch.arange(gflat.numel(), dtype=torch.float32) * (rank + 1)
        early = D.allreduce_mean_async_(g2[split:], bucket_bytes=64)
        late = D.allreduce_mean_async_(g2[:split], bucket_bytes=64)
        D.finish_allreduce_(early)
        D.finish_allreduce_(late)
        torch.testing.assert_close(g2, torch.arange(gflat.numel(), dtype=torch.float32) * 1.5)
        q.put((rank, flat.clone(), gflat.clone(), m[0].weight.grad.clone()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surface worker failures to the parent
        q.put((rank, repr(e), None, None))
        raise


@pytest.mark.timeout(120)
def test_dp_broadcast_and_allreduce_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        rank, flat, gflat, g0 = q.get(timeout=100)
        assert not isinstance(flat, str), flat
        res[rank] = (flat, gflat, g0)
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    torch.testing.assert_close(res[0][0], res[1][0], rtol=0, atol=0)  # weights identical after broadcast
    n = res[0][1].numel()
    expect = torch.arange(n, dtype=torch.float32) * 1.5  # mean of (1x, 2x)
    for r in (0, 1):
        torch.testing.assert_close(res[r][1], expect)
        torch.testing.assert_close(res[r][2].reshape(-1), expect[:35])  # .grad views the flat buffer (offset 0)


def test_single_process_is_a_noop(monkeypatch):
    from autoformer_amd import dist as D

    monkeypatch.setenv("WORLD_SIZE", "1")
    assert D.init_from_env("gloo") == (0, 1, 0)
    g = torch.ones(10)
    D.allreduce_mean_(g)
    D.broadcast_(g)
    assert torch.equal(g, torch.ones(10))


def test_recurrence_launch_refused_while_collective_outstanding():
    """DESIGN §6 invariant: no persistent (decoder, H > 64) recurrence is enqueued while an RCCL
    collective is outstanding on the comm stream (its polling kernels can hold the CU slots the
    recurrence's whole grid needs).  The host check fires before any device work."""
    from autoformer_amd import kernels as K

    K.collective_joined()
    K.collective_enqueued("decoder-slice all-reduce")
    try:
        for fn, args in ((K.lstm2_fwd, (None,) * 5 + (64, 128, 1024)),
                         (K.lstm2_bwd, (None,) * 8 + (64, 128, 1024)),
                         (K.lstm_fwd, (None, None, 64, 128, 512, 1)),
                         (K.lstm_bwd, (None,) * 6 + (64, 128, 512, 1))):
            with pytest.raises(RuntimeError, match="outstanding"):
                fn(*args)
        assert K.collectives_outstanding() == ["decoder-slice all-reduce"]
    finally:
        K.collective_joined()
    assert not K.collectives_outstanding()
