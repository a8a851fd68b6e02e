"""Data parallelism for the training step: one process per GPU, utterance batches sharded
across ranks, per-replica BatchNorm (no SyncBN — the reference is single-device and
its BN statistics are per batch of 64), gradients averaged with one
bucketed all-reduce over the flat gradient buffer (RCCL over xGMI when the backend is
"nccl"; gloo on CPU for tests).

The reference has no distributed code at all; this is the only exchange
step of the path.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

BUCKET_BYTES = 32 << 20


def init_from_env(backend: str = "nccl"):
    """Initialise the default process group from torchrun's env; returns (rank, world, local_rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 0, 1, 0
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if not dist.is_initialized():
        dist.init_process_group(backend=backend)
    return dist.get_rank(), dist.get_world_size(), int(os.environ.get("LOCAL_RANK", "0"))


PARAM_ALIGN = 64  # elements (256 B): every parameter view starts on a 16-B multiple, so the
                  # GEMMs' vectorised (buffer-load / LDS-DMA) operand paths accept it in place


def param_offsets(params):
    """Start offset of each parameter in the flat buffer and the buffer length."""
    offs, off = [], 0
    for p in params:
        offs.append(off)
        off += -(-p.numel() // PARAM_ALIGN) * PARAM_ALIGN
    return offs, off


def flatten_params_(module, device=None):
    """Move every parameter into one contiguous fp32 buffer (and its .grad into another)
    so the optimizer and the all-reduce are single kernels over 28.5M values.  Each view
    starts PARAM_ALIGN-aligned; the few padding elements stay zero (zero gradient, so Adam
    leaves them at zero).  Returns (params, flat, gflat)."""
    params = [p for p in module.parameters() if p.requires_grad]
    device = device or params[0].device
    offs, n = param_offsets(params)
    flat = torch.zeros(n, device=device, dtype=torch.float32)
    gflat = torch.zeros(n, device=device, dtype=torch.float32)
    with torch.no_grad():
        for p, off in zip(params, offs):
            k = p.numel()
            flat[off:off + k].copy_(p.detach().reshape(-1))
            p.data = flat[off:off + k].view_as(p)
            p.grad = gflat[off:off + k].view_as(p)
    return params, flat, gflat


def broadcast_(flat: torch.Tensor, src: int = 0):
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast(flat, src)


def allreduce_mean_async_(g: torch.Tensor, bucket_bytes: int = BUCKET_BYTES):
    """Start averaging `g` over ranks in ~32 MB buckets (xGMI ring: per-link bound, so a few
    large collectives beat many small ones).  Returns a handle for finish_allreduce_()."""
    if not (dist.is_initialized() and dist.get_world_size() > 1) or g.numel() == 0:
        return None
    use_avg = dist.get_backend() == "nccl"
    step = max(1, bucket_bytes // g.element_size())
    works = [dist.all_reduce(g[off:off + step], op=dist.ReduceOp.AVG if use_avg else dist.ReduceOp.SUM,
                             async_op=True) for off in range(0, g.numel(), step)]
    return works, g, use_avg


def finish_allreduce_(handle):
    """Wait for allreduce_mean_async_ (RCCL: the current stream waits on the collective)."""
    if handle is None:
        return
    works, g, use_avg = handle
    for w in works:
        w.wait()
    if not use_avg:
        g.mul_(1.0 / dist.get_world_size())


def allreduce_mean_(gflat: torch.Tensor, bucket_bytes: int = BUCKET_BYTES):
    """Average gradients over ranks (blocking form of allreduce_mean_async_)."""
    finish_allreduce_(allreduce_mean_async_(gflat, bucket_bytes))


def split_offset(params, first_late):
    """Flat-buffer offset where parameter `first_late` (in flatten_params_ order) starts: the
    gradients below it (the encoder, used by both the full pass and the re-pass) complete last,
    the ones from it on (decoder, postnet, discriminator) are final before the encoder
    backward runs and are all-reduced while it runs."""
    offs, _ = param_offsets(params)
    for p, off in zip(params, offs):
        if p is first_late:
            return off
    raise ValueError("parameter not in the flattened list")
