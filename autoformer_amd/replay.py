"""Recorded-step replay: the host side of a training step reduced to a list of native calls.

Eager, a C2 step spends ~5 ms of Python (autograd, the layer wrappers, descriptor building,
ctypes) to queue ~5.7 ms of GPU work: on a slow-host box the GPU waits for the host.  A hipGraph
removes the host but the runtime serialises the weight-gradient side stream inside it or pays
15-100 us at every cut between graph segments (profiles/r5_graph_modes.txt).  This
module records ONE step as the exact sequence of library entry points it made (function, frozen
arguments: every pointer, shape, stream and event handle) and replays that sequence: the same
kernels on the same two streams with the same event edges as the eager step -- the side stream
still runs beside the main chain -- with none of the Python that produced them.

What makes a recorded argument list valid again at the next step:
  * every tensor the step allocates (each aten allocation is seen by the dispatch mode below) is
    held by the record, so no address frozen in the calls is ever freed or handed to anything else
    -- not within the step either, so the recording step's buffers are all distinct and no
    cross-stream reuse hazard exists in the replays (a private MemPool had been used first: its
    freed blocks were taken by other allocations of the process, tests/test_gpu_replay.py with an
    eager trainer beside the replaying one);
  * weight packs are frozen and rewritten in place after the optimizer step inside the recorded
    step (layers.freeze_packs / repack_in_place, as for the captured graph);
  * device-side state (Adam's step count, BN running statistics, the LSTM hand-off flags and
    last-arrival counters) already lives on the device and advances in the kernels themselves.
Torch operations issued inside the step (the gradient buffer's zero fill, autograd's own glue)
are caught by a dispatch mode while recording and replayed as closures over the same tensors: an
in-place op is re-run as it is, an out-of-place one recomputes into the tensor it returned.
`StepRecord.torch_ops` lists them (the C2 step: the zero fill and four autograd gradient sums).

The data-parallel gradient average (RCCL) is not a library call: TrainStep issues it through
collective(), which the replay re-runs at its place on its stream.  A replay needs the same input
tensors at every step (TrainStep.record copies a new batch into them), as a graph does."""
from __future__ import annotations

import contextlib
import ctypes

import torch
from torch.utils._python_dispatch import TorchDispatchMode
from torch.utils._pytree import tree_flatten

from . import _lib as L

# aten ops that launch no kernel (allocation, metadata, host reads)
_NO_KERNEL = {"empty", "empty_strided", "empty_like", "new_empty", "new_empty_strided", "_local_scalar_dense",
              "record_stream", "resize_", "set_", "lift_fresh", "detach", "is_same_size", "sym_size",
              "sym_stride", "sym_numel", "sym_storage_offset", "_has_compatible_shallow_copy_type"}


def _cuda_tensors(args, kwargs):
    flat, _ = tree_flatten((args, kwargs))
    return any(isinstance(t, torch.Tensor) and t.is_cuda for t in flat)


def _copy_into(dst, src):
    if isinstance(dst, torch.Tensor):
        dst.copy_(src)
    elif isinstance(dst, (tuple, list)):
        for d, s in zip(dst, src):
            _copy_into(d, s)


class _TorchOpRecorder(TorchDispatchMode):
    def __init__(self, rec):
        super().__init__()
        self.rec = rec

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        out = func(*args, **kwargs)
        if not self.rec.paused:
            # every device tensor the step allocates stays allocated while the record lives: the
            # addresses frozen in the calls can never be handed to anything else
            flat, _ = tree_flatten(out)
            self.rec.keep.extend(t for t in flat if isinstance(t, torch.Tensor) and t.is_cuda)
        if (self.rec.paused or func.is_view or func.overloadpacket.__name__ in _NO_KERNEL
                or not _cuda_tensors(args, kwargs)):
            return out
        outf = getattr(func.overloadpacket, "out", None) if isinstance(out, torch.Tensor) else None
        if func._schema.is_mutable:
            def run(func=func, args=args, kwargs=kwargs):
                func(*args, **kwargs)
        elif outf is not None:
            # autograd's gradient sums (aten.add) and the like: the op's .out form into the tensor
            # the recording returned (no allocation, no copy)
            def run(outf=outf, args=args, kwargs=kwargs, out=out):
                outf(*args, **kwargs, out=out)
        else:
            def run(func=func, args=args, kwargs=kwargs, out=out):
                _copy_into(out, func(*args, **kwargs))
        self.rec.calls.append((None, run, None))
        self.rec.torch_ops.append(str(func))
        return out


def _frozen(a):
    """A recorded argument: ctypes structures are copied (the caller may reuse its object)."""
    if isinstance(a, ctypes.Structure):
        return type(a).from_buffer_copy(a)
    return a


class StepRecord:
    """The recorded calls of one step; replay() re-issues them.  Keeps every device tensor the
    recorded step allocated (and every tensor a torch-op closure references) alive."""

    def __init__(self):
        self.calls = []       # (ctypes function, name, args) | (None, closure, None)
        self.torch_ops = []   # names of the torch ops recorded as closures
        self.keep = []
        self.paused = False   # inside collective(): nothing is recorded call by call

    def native_calls(self):
        return sum(1 for c in self.calls if c[0] is not None)

    def add_native(self, fn, name, args):
        self.calls.append((fn, name, tuple(_frozen(a) for a in args)))

    def add_marker(self, closure):
        """A host closure run at this point of every replay (e.g. a timing event record)."""
        self.calls.append((None, closure, None))

    def replay(self):
        check = L.check
        with torch.no_grad():  # the torch-op closures write into tensors that may require grad
            for fn, name, args in self.calls:
                if fn is None:
                    name()
                    continue
                rc = fn(*args)
                if rc:
                    check(rc, name)


def collective(fn):
    """Run fn() (a torch.distributed collective and its wait, issued on the current stream); inside a
    recording, every replay re-runs fn at this point on the same stream instead of recording what
    it issues (the RCCL launch is not a library call).  Returns fn's result."""
    rec = L._REC
    if rec is None:
        return fn()
    stream = torch.cuda.current_stream()
    rec.paused, L._REC = True, None
    try:
        out = fn()
    finally:
        rec.paused, L._REC = False, rec

    def run():
        with torch.cuda.stream(stream):
            fn()
    rec.add_marker(run)
    return out


@contextlib.contextmanager
def recording(rec: StepRecord):
    """Record every library call (and torch op) issued inside the block into `rec`, holding every
    device tensor allocated inside it; autograd runs its backward on this thread so that the
    dispatch mode sees it too."""
    if L._REC is not None:
        raise RuntimeError("replay.recording: already recording")
    mt = torch.autograd.is_multithreading_enabled()
    torch.autograd.set_multithreading_enabled(False)
    L._REC = rec
    try:
        with _TorchOpRecorder(rec):
            yield rec
    finally:
        L._REC = None
        torch.autograd.set_multithreading_enabled(mt)
