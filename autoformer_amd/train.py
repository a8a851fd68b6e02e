"""Training drivers: the reference Solver step re-expressed over HIP kernels.

* ``Solver`` mirrors /root/reference/train.py:13-132 (same constructor, same loop, same
  losses and logging format) so existing scripts can switch by import.
* ``GANSolver`` mirrors train_with_discriminator.py:13-145 (ONE loss for both models and
  both Adams stepping on the same backward — kept as in the reference, not "fixed"); the
  benchmark form of the same step is ``TrainStep(G, extra=gan_extra(D), extra_modules=[D])``.
* ``AdjustSolver`` mirrors train_with_adjust.py:16-145 (the *_Adjust models, 4 losses).
* ``TrainStep`` is the benchmark/production step: flat parameter and gradient buffers,
  HIP MSE/L1 losses, fused HIP Adam, optional RCCL gradient all-reduce and hipGraph
  capture of the whole step.

Step semantics (train.py:82-99): full forward, MSE(x, mel) + MSE(x, mel_postnet),
encoder re-pass on mel_postnet, L1(codes, codes_re), sum (lambda_cd = 1), zero_grad,
backward, Adam(lr = 1e-4, betas (0.9, 0.999), eps 1e-8).
"""
from __future__ import annotations

import datetime
import importlib
import os
import time

import torch

from . import dist as D
from . import kernels as K
from .replay import collective
from .layers import (ev_record, freeze_packs, join_side, on_stream, plan_caches, prefetch_packs,
                     repack_in_place, set_grad_sink, set_tail, side_stream, stream_wait,
                     weights_changed)


def _load_state(model, path, device):
    """torch.load(path, map_location=device) into model (train_with_adjust.py:50-54); a
    tensors-only loader (weights_only) -- a state_dict needs nothing else."""
    model.load_state_dict(torch.load(path, map_location=device, weights_only=True))


# ------------------------------------------------------------------------- losses
class _MSEFn(torch.autograd.Function):
    """F.mse_loss(a, b), mean reduction (train.py:85-86)."""

    @staticmethod
    def forward(ctx, a, b):
        a, b = a.contiguous(), b.contiguous()
        ctx.save_for_backward(a, b)
        return K.mse_loss(a, b)

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        g = g.contiguous()
        ga = K.loss_grad(a, b, g, 0, 1.0) if ctx.needs_input_grad[0] else None
        gb = K.loss_grad(a, b, g, 0, -1.0) if ctx.needs_input_grad[1] else None
        return ga, gb


class _L1Fn(torch.autograd.Function):
    """F.l1_loss(a, b), mean reduction (train.py:94)."""

    @staticmethod
    def forward(ctx, a, b):
        a, b = a.contiguous(), b.contiguous()
        ctx.save_for_backward(a, b)
        return K.l1_loss(a, b)

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        g = g.contiguous()
        ga = K.loss_grad(a, b, g, 1, 1.0) if ctx.needs_input_grad[0] else None
        gb = K.loss_grad(a, b, g, 1, -1.0) if ctx.needs_input_grad[1] else None
        return ga, gb


class _BCEFn(torch.autograd.Function):
    """nn.BCELoss(mean) against a constant target (train_with_discriminator.py:58-61)."""

    @staticmethod
    def forward(ctx, p, target):
        p = p.contiguous()
        ctx.save_for_backward(p)
        ctx.target = float(target)
        return K.bce_loss(p, target)

    @staticmethod
    def backward(ctx, g):
        (p,) = ctx.saved_tensors
        return K.bce_grad(p, ctx.target, g.contiguous()), None


def bce_loss(p, target):
    return _BCEFn.apply(p, target)


def discriminator_loss(real, fake):
    """train_with_discriminator.py:58-61."""
    return bce_loss(real, 1.0) + bce_loss(fake, 0.0)


def gan_extra(D):
    """Extra loss term of the two-model step (train_with_discriminator.py:102-107):
    d_loss = BCE(D(x_real), 1) + BCE(D(x_identic_psnt.squeeze()), 0), added to the G loss."""
    def extra(x_real, emb, x_psnt):
        return discriminator_loss(D(x_real), D(x_psnt.squeeze()))
    return extra


class _VCLossFn(torch.autograd.Function):
    """The loss block of Solver.train (train.py:84-96) as one launch forward and one backward:
    (total, l_id, l_id_psnt, l_cd) with total = l_id + l_id_psnt + lambda_cd * l_cd, where
    l_id = F.mse_loss(x_real, x_identic), l_id_psnt = F.mse_loss(x_real, x_identic_psnt),
    l_cd = F.l1_loss(code_real, code_reconst).  The separate losses' kernels, their zeroing
    memsets and the scalar adds / multiply of the reference's expression are gone; the upstream
    gradients of all four outputs reach the one gradient kernel as device scalars."""

    @staticmethod
    def forward(ctx, x, y1, y2, ca, cb, lambda_cd):
        x, y1, y2 = x.contiguous(), y1.reshape(x.shape).contiguous(), y2.reshape(x.shape).contiguous()
        ca, cb = ca.contiguous(), cb.reshape(ca.shape).contiguous()
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(x, y1, y2, ca, cb)
        ctx.lam = float(lambda_cd)
        out = K.vc_loss(x, y1, y2, ca, cb, ctx.lam)
        return out[3], out[0], out[1], out[2]

    @staticmethod
    def backward(ctx, d_total, d_id, d_psnt, d_cd):
        x, y1, y2, ca, cb = ctx.saved_tensors
        need = ctx.needs_input_grad
        d = [t.contiguous() if t is not None else None for t in (d_id, d_psnt, d_cd, d_total)]
        # a term whose upstream gradients are all None contributes nothing (None, not zeros);
        # x_real is data in train.py, its gradient (rare) is -(g1 + g2)
        t = d_total is not None
        h1, h2, hc = t or d_id is not None, t or d_psnt is not None, t or d_cd is not None
        n1, n2 = h1 and (need[1] or need[0]), h2 and (need[2] or need[0])
        want = (n1, n2, hc and need[3], hc and need[4])
        if not any(want):
            return None, None, None, None, None, None
        g1, g2, ga, gb = K.vc_loss_grad(x, y1, y2, ca, cb, ctx.lam, d, want)
        gx = None
        if need[0] and (g1 is not None or g2 is not None):
            gx = -(g1 + g2) if g1 is not None and g2 is not None else -(g1 if g1 is not None else g2)
        return gx, g1 if need[1] else None, g2 if need[2] else None, ga, gb, None


def vc_loss_block(x_real, x_id, x_id_psnt, code_real, code_re, lambda_cd=1.0):
    """(total, (l_id, l_id_psnt, l_cd)) of train.py:84-96, fused (_VCLossFn)."""
    total, l_id, l_psnt, l_cd = _VCLossFn.apply(x_real, x_id, x_id_psnt, code_real, code_re, lambda_cd)
    return total, (l_id, l_psnt, l_cd)


def mse_loss(a, b):
    return _MSEFn.apply(a, b.reshape(a.shape))


def l1_loss(a, b):
    return _L1Fn.apply(a, b.reshape(a.shape))


def vc_losses(model, x_real, emb, lambda_cd=1.0):
    """The loss block of Solver.train (train.py:84-96)."""
    x_id, x_id_psnt, code_real = model(x_real, emb, emb)
    code_re = model(x_id_psnt, emb, None)
    total, parts = vc_loss_block(x_real, x_id.squeeze(), x_id_psnt.squeeze(), code_real, code_re, lambda_cd)
    return total, parts, x_id_psnt


def adain_losses(model, x_real, emb, lambda_cd=1.0):
    """train.py's loss block with isadain=True (train.py:89-92) for the AdaIN variants
    (AutoVC2 & co.), whose c_trg=None pass returns (codes, features) (AutoVC2.py:219-220)."""
    x_id, x_id_psnt, code_real = model(x_real, emb, emb)
    code_re, _ = model(x_id_psnt, emb, None)
    total, parts = vc_loss_block(x_real, x_id.squeeze(), x_id_psnt.squeeze(), code_real, code_re, lambda_cd)
    return total, parts, x_id_psnt


def adjust_losses(model, x_real, emb, lambda_cd=1.0, lambda_ad=1.0):
    """The loss block of train_with_adjust.py:Solver.train (train_with_adjust.py:96-124)."""
    emb_adjust, x_id, x_id_psnt, code_real = model(x_real, emb, emb)
    code_re = model(x_id_psnt, emb, None)
    total, (l_id, l_id_psnt, l_cd) = vc_loss_block(x_real, x_id.squeeze(), x_id_psnt.squeeze(), code_real, code_re,
                                                   lambda_cd)
    l_ad = l1_loss(emb_adjust, emb)
    return (total + lambda_ad * l_ad, (l_id, l_id_psnt, l_cd, l_ad), x_id_psnt)


def losses_for(model):
    """The step's loss block by model family (plain / AdaIN variant / Adjust variant)."""
    from .factory._variants import AdaINModel, AdjustModel

    if isinstance(model, AdjustModel):
        return adjust_losses
    if isinstance(model, AdaINModel):
        return adain_losses
    return vc_losses


# ------------------------------------------------------------------------- optimizer
class FusedAdam:
    """torch.optim.Adam (defaults, no weight decay) as one HIP kernel over a flat buffer."""

    def __init__(self, flat, gflat, lr=1e-4, betas=(0.9, 0.999), eps=1e-8):
        self.flat, self.gflat = flat, gflat
        self.lr, self.betas, self.eps = lr, betas, eps
        self.m = torch.zeros_like(flat)
        self.v = torch.zeros_like(flat)
        self.state = torch.zeros(4, device=flat.device)

    def zero_grad(self):
        self.gflat.zero_()

    def step(self):
        K.adam(self.flat, self.gflat, self.m, self.v, self.lr, self.betas[0], self.betas[1], self.eps, self.state)
        weights_changed()

    def step_slice(self, lo, hi, advance, max_blocks=0):
        """Adam over flat[lo:hi] only; `advance` on the step's first slice (the step count and
        bias corrections live in self.state; later slices must be stream-ordered after it).
        max_blocks: workgroup cap for a slice that runs beside other kernels."""
        sl = slice(lo, hi)
        K.adam(self.flat[sl], self.gflat[sl], self.m[sl], self.v[sl], self.lr, self.betas[0], self.betas[1],
               self.eps, self.state, advance=advance, max_blocks=max_blocks)


# ------------------------------------------------------------------------- bench step
# workgroup cap of the decoder-slice Adam that runs beside the encoder backward (0 = full grid: it slowed
# the latency-bound BiLSTM backward beside it; 64 / 24 let the step's tail wait for it,
# profiles/r5_replay_ab.txt).  Round 6, with the 16-B vector Adam: 512 (5.654 / 5.647 ms) vs 256 (5.683 /
# 5.661), 128 (5.682 / 5.665), 1024 (5.667 / 5.693), profiles/r6_pack_ab.txt
_SIDE_ADAM_BLOCKS = 512


class TrainStep:
    """One train.py step over the HIP model with flat buffers, optional DP and a recorded replay.

    With world > 1 the gradients are averaged by RCCL between backward and Adam; after
    `record()` every step replays the recorded native calls (replay.py), the collectives included."""

    def __init__(self, model, lr=1e-4, lambda_cd=1.0, extra=None, extra_modules=()):
        self.model = model
        self.lambda_cd = lambda_cd
        self.extra = extra  # optional callable(x, emb, x_psnt) -> extra loss (GAN step)
        # one flat buffer (and one fused Adam) over every module: Adam is elementwise, so this
        # equals the reference's separate g_optimizer / d_optimizer with the same settings.  The
        # extra modules (the GAN step's discriminator) go FIRST, below the split offset: their
        # gradients (the real-data branch D(x) included) are complete only at the end of the
        # backward, not when the decoder hook fires, so they are stepped with the encoder slice
        owner = torch.nn.ModuleList([*extra_modules, model]) if extra_modules else model
        self.params, self.flat, self.gflat = D.flatten_params_(owner)
        D.broadcast_(self.flat)
        set_grad_sink(True)  # kernels accumulate straight into the flat gradient buffer
        self.opt = FusedAdam(self.flat, self.gflat, lr)
        self.world = torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1
        self.loss = None
        # The decoder / postnet (/ discriminator) gradients are final once the backward reaches
        # the decoder input (encoder parameters precede them in the flat buffer).  From that
        # point, on a second stream and beside the encoder backward (full pass + re-pass, the
        # latency-bound BiLSTM recurrences), their slice is averaged over ranks (data parallel)
        # and stepped by Adam; after the backward only the encoder slice (13 %) is left.
        self.split = None
        self.loss_fn = losses_for(model)
        # the Adjust variants register `adjust` after the postnet and its gradients complete
        # only with the encoder's: no early (overlapped) slice for them
        if hasattr(model, "decoder") and self.loss_fn is not adjust_losses:
            self.split = D.split_offset(self.params, next(model.decoder.parameters()))
            self.comm = torch.cuda.Stream()
        self._early = None
        self._early_adam = False
        self._recording = False  # inside record(): the decoder's weight packs are rewritten in place
        self._pack_groups = None  # (encoder-slice caches, decoder-slice caches) of a recorded step
        # fault word (kernels.fault_word): read back asynchronously after every step into a
        # pinned word and checked at the next step, so a failed persistent recurrence raises
        # within one step without a host sync; check() is the synchronous form
        self._fault = K.fault_word(self.flat.device)
        self._fault_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self._fault_ev = None
        self._one = torch.ones((), device=self.flat.device)
        self.recorded = None  # replay.StepRecord of record(): step() replays it
        # optional exposed all-reduce time: a list of (start, end) HIP event pairs recorded on
        # the main stream around its wait for the collective (bench.py's allreduce_ms)
        self.comm_timing = None

    def _probe_fault(self):
        if self._fault_ev is not None and self._fault_ev.query():
            K.raise_on_fault(self._fault_host.item())
        comm = getattr(self, "comm", None)
        if comm is not None:
            # the read-back copy and its event on the comm stream, behind the step's main-stream work: the
            # main stream records one event instead of running the copy and a fenced event itself
            stream_wait(comm.cuda_stream, ev_record())
            with on_stream(comm):
                self._fault_host.copy_(self._fault, non_blocking=True)
                self._fault_ev = torch.cuda.Event()
                self._fault_ev.record(comm)
            return
        self._fault_host.copy_(self._fault, non_blocking=True)
        self._fault_ev = torch.cuda.Event()
        self._fault_ev.record()

    def check(self):
        """Raise DeviceFault if any kernel of the steps so far reported a fault (synchronises)."""
        torch.cuda.synchronize()
        K.raise_on_fault(self._fault.item())

    def _decoder_done(self):
        set_tail(True)  # the rest of the backward is the encoder's full pass (layers.main_wgrad)
        comm = self.comm.cuda_stream
        stream_wait(comm, ev_record())
        side = side_stream()
        if side is not None:
            stream_wait(comm, ev_record(side.cuda_stream))
        with on_stream(self.comm):
            if self.world > 1:
                # RCCL: the comm stream waits for the collective; the Adam slice follows it
                g = self.gflat[self.split:]
                collective(lambda: D.finish_allreduce_(D.allreduce_mean_async_(g)))
                K.collective_enqueued("decoder-slice all-reduce")
            self.opt.step_slice(self.split, self.flat.numel(), advance=True, max_blocks=_SIDE_ADAM_BLOCKS)
            if self._recording:
                # recorded step: the decoder's weight packs rewritten in place right after its Adam
                # slice, on this stream (the next step's forward is ordered after it by the tail's wait)
                repack_in_place(self._pack_groups[1], "graph_dec")
        self._early_adam = True

    def _fwd_bwd(self, x, emb, overlap=False):
        self.gflat.zero_()
        self.model._decoder_bwd_done = self._decoder_done if overlap else None
        try:
            loss, parts, x_psnt = self.loss_fn(self.model, x, emb, self.lambda_cd)
            if self.extra is not None:
                loss = loss + self.extra(x, emb, x_psnt)
            # the seed gradient is a persistent tensor: backward() alone would allocate and fill
            # a ones_like per step (one more kernel, and a closure in a recorded step)
            loss.backward(self._one if loss.dim() == 0 else None)
        finally:
            self.model._decoder_bwd_done = None
        join_side()  # weight-gradient GEMMs ran on the side stream
        return loss

    def _finish(self):
        """After the backward: average what is left over ranks and run Adam on it."""
        timed = self.comm_timing is not None and self.world > 1
        if timed:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        if not self._early_adam:  # no overlapped part (no decoder hook fired)
            if self.world > 1:
                D.allreduce_mean_(self.gflat)
            if timed:
                ev[1].record()
            self.opt.step()
        else:
            if self.world > 1:
                self.comm.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(self.comm):
                    D.finish_allreduce_(D.allreduce_mean_async_(self.gflat[:self.split]))
                K.collective_enqueued("encoder-slice all-reduce")
            stream_wait(K.stream(), ev_record(self.comm.cuda_stream))  # the early slice's Adam (and its step count)
            K.collective_joined()
            if timed:
                ev[1].record()
            self.opt.step_slice(0, self.split, advance=False)
            weights_changed()
            self._early, self._early_adam = None, False
        if timed:
            self.comm_timing.append(ev)

    def step(self, x, emb):
        return self._step(x, emb)

    def _step(self, x, emb):
        if self.recorded is not None:
            # the recorded step's native calls, re-issued without the Python that made them: the
            # same kernels on the same main / side streams and event edges (replay.py)
            if x is not self._rx:
                self._rx.copy_(x)
            if emb is not self._re:
                self._re.copy_(emb)
            self.recorded.replay()
            self._probe_fault()
            return self.loss
        loss = self._fwd_bwd(x, emb, overlap=self.split is not None)
        self._finish()
        prefetch_packs()  # next step's weight packs, on the side stream
        self._probe_fault()
        return loss

    def _freeze_pack_groups(self):
        """Split the live weight packs into the encoder / decoder slices' groups and bring their
        in-place op tables and contents up to date (eager); the caller then freezes them."""
        bound = self.flat[self.split].data_ptr() if self.split is not None else None
        dec = (lambda c: c.params[0].data_ptr() >= bound) if bound is not None else (lambda c: False)
        # only this trainer's packs (the plan is process-wide: another model's caches would be frozen
        # into this step's repack and rewritten through pointers that model may free later)
        lo = self.flat.data_ptr()
        hi = lo + self.flat.numel() * self.flat.element_size()
        own = lambda c: lo <= c.params[0].data_ptr() < hi  # noqa: E731
        self._pack_groups = (plan_caches(lambda c: own(c) and not dec(c)), plan_caches(lambda c: own(c) and dec(c)))
        for caches, grp in ((self._pack_groups[0], "graph_enc"), (self._pack_groups[1], "graph_dec"),
                            (self._pack_groups[0] + self._pack_groups[1], "graph_all")):
            repack_in_place(caches, grp)  # eager: builds the op tables (and the current packs)

    def _recordable_tail(self):
        """The optimizer step + in-place weight repack that end a recorded step (with the gradient
        average over ranks first when world > 1)."""
        if self._early_adam:  # the decoder slice's average + Adam + repack ran on the comm stream
            comm = self.comm.cuda_stream
            if self.world > 1:
                box = self._comm_timing_mark(None)
                stream_wait(comm, ev_record())
                g = self.gflat[:self.split]
                with on_stream(self.comm):
                    collective(lambda: D.finish_allreduce_(D.allreduce_mean_async_(g)))
                K.collective_enqueued("encoder-slice all-reduce")
            stream_wait(K.stream(), ev_record(comm))
            K.collective_joined()
            if self.world > 1:
                self._comm_timing_mark(box)
            self.opt.step_slice(0, self.split, advance=False)
            repack_in_place(self._pack_groups[0], "graph_enc")
        else:
            if self.world > 1:
                collective(lambda: D.allreduce_mean_(self.gflat))
            K.adam(self.flat, self.gflat, self.opt.m, self.opt.v, self.opt.lr, self.opt.betas[0],
                   self.opt.betas[1], self.opt.eps, self.opt.state)
            repack_in_place(self._pack_groups[0] + self._pack_groups[1], "graph_all")

    def _comm_timing_mark(self, box):
        """Recorded step: a marker that brackets the main stream's wait for the gradient average with
        HIP events whenever comm_timing is a list at replay (bench.py's allreduce_ms); box=None
        starts a bracket and returns it, a box closes it."""
        from . import _lib as L

        s = torch.cuda.current_stream()
        if box is None:
            box = []

            def start():
                if self.comm_timing is not None:
                    box[:] = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))]
                    box[0][0].record(s)
            L._REC.add_marker(start)
            return box

        def end():
            if self.comm_timing is not None and box:
                box[0][1].record(s)
                self.comm_timing.append(box.pop())
        L._REC.add_marker(end)
        return box

    def replayable(self):
        """Whether record() applies (every TrainStep; kept for callers that probe it)."""
        return True

    def record(self, x, emb, warmup=2):
        """Run one step while recording its native calls (replay.py); every later step() replays
        them: the whole step (zero_grad, forward, re-pass, losses, backward with the weight-gradient
        side stream, both Adam slices, the in-place weight repack) with no Python per kernel.
        x, emb become the step's input buffers: step() with other tensors copies them in.  With
        world > 1 the gradient average (RCCL) is re-issued at its place by replay.collective."""
        from . import replay as R

        for _ in range(warmup):
            self.step(x, emb)
        torch.cuda.synchronize()
        weights_changed()
        self._freeze_pack_groups()
        torch.cuda.synchronize()
        freeze_packs(True)
        # the decoder slice's Adam beside the encoder backward (comm stream), as in the eager step
        # (a high-priority stream for the recorded main chain and a single Adam after the backward
        # measured no better: profiles/r5_replay_ab.txt)
        self._recording = self.split is not None
        rec = R.StepRecord()
        try:
            with R.recording(rec):
                self.loss = self._fwd_bwd(x, emb, overlap=self._recording)
                self._recordable_tail()
        finally:
            self._recording = False
            self._early_adam = False
            freeze_packs(False)
        weights_changed()
        self._probe_fault()
        self.recorded, self._rx, self._re = rec, x, emb
        return rec


# ------------------------------------------------------------------------- reference-shaped solvers
class Solver:
    """Mirror of train.py:Solver (train.py:13-132) on the HIP model; torch.optim.Adam is
    replaced by FusedAdam over flat buffers, losses by the HIP loss kernels."""

    def __init__(self, vcc_loader, config):
        self.vcc_loader = vcc_loader
        self.lambda_cd = config.lambda_cd
        self.dim_neck, self.dim_emb = config.dim_neck, config.dim_emb
        self.dim_pre, self.freq = config.dim_pre, config.freq
        self.isadain = getattr(config, "isadain", False)
        self.model_name = config.model_name
        self.batch_size, self.num_iters = config.batch_size, config.num_iters
        self.device = config.device
        self.log_step = config.log_step
        self.build_model()

    def build_model(self):
        self.VC = getattr(importlib.import_module(f"autoformer_amd.factory.{self.model_name}"), self.model_name)(
            self.dim_neck, self.dim_emb, self.dim_pre, self.freq)
        if getattr(self, "use_pretrained_weight", False):
            print(f"Load Pre-trained Weight --- {self.pretrained_weight_path}")
            _load_state(self.VC, self.pretrained_weight_path, self.device)
        self.VC.to(self.device)
        _, flat, gflat = D.flatten_params_(self.VC)
        self.vc_optimizer = FusedAdam(flat, gflat, 0.0001)

    def _optimize(self, loss):
        """reset_grad; backward; Adam (train.py:97-99).  The weight-gradient kernels may still be
        writing .grad on the side stream (gradient-sink mode): join it before Adam reads it."""
        self.reset_grad()
        loss.backward()
        join_side()
        self.vc_optimizer.step()

    def _read(self, keys, parts):
        """loss.item() of each term (train.py:103-105) plus the device fault check."""
        loss = {k: p.item() for k, p in zip(keys, parts)}
        K.check_faults(parts[0].device)
        return loss

    def reset_grad(self):
        self.vc_optimizer.zero_grad()

    def train(self):
        keys = ["VC/loss_id", "VC/loss_id_psnt", "VC/loss_cd"]
        print("Start training...")
        start_time = time.time()
        data_iter = None
        history = []
        for i in range(self.num_iters):
            try:
                x_real, emb_org = next(data_iter)
            except Exception:
                data_iter = iter(self.vcc_loader)
                x_real, emb_org = next(data_iter)
            x_real = x_real.to(self.device)
            emb_org = emb_org.to(self.device)
            self.VC = self.VC.train()
            # train.py:89-92: with isadain the re-pass returns (codes, features)
            step_losses = adain_losses if self.isadain else vc_losses
            vc_loss, parts, _ = step_losses(self.VC, x_real, emb_org, self.lambda_cd)
            self._optimize(vc_loss)
            loss = self._read(keys, parts)
            history.append([loss[k] for k in keys])
            if (i + 1) % self.log_step == 0:
                et = str(datetime.timedelta(seconds=time.time() - start_time))[:-7]
                log = "Elapsed [{}], Iteration [{}/{}]".format(et, i + 1, self.num_iters)
                for tag in keys:
                    log += ", {}: {:.4f}".format(tag, loss[tag])
                print(log)
        return history


class AdjustSolver(Solver):
    """Mirror of train_with_adjust.py:Solver (train_with_adjust.py:16-145): the train.py loop
    plus the speaker-embedding loss L1(emb_adjust, emb_org) weighted by lambda_ad."""

    def __init__(self, vcc_loader, config):
        self.lambda_ad = getattr(config, "lambda_ad", 1.0)
        # train_with_adjust.py:32-33,50-54 (the flag is bool(str) there: any non-empty string)
        self.use_pretrained_weight = bool(getattr(config, "use_pretrained_weight", False))
        self.pretrained_weight_path = getattr(config, "pretrained_weight_path", None)
        super().__init__(vcc_loader, config)

    def train(self):
        keys = ["G/loss_id", "G/loss_id_psnt", "G/loss_cd", "A/loss_adjust"]
        print("Start training...")
        start_time = time.time()
        data_iter = None
        history = []
        for i in range(self.num_iters):
            try:
                x_real, emb_org = next(data_iter)
            except Exception:
                data_iter = iter(self.vcc_loader)
                x_real, emb_org = next(data_iter)
            x_real = x_real.to(self.device)
            emb_org = emb_org.to(self.device)
            self.VC = self.VC.train()
            g_loss, parts, _ = adjust_losses(self.VC, x_real, emb_org, self.lambda_cd, self.lambda_ad)
            self._optimize(g_loss)
            loss = self._read(keys, parts)
            history.append([loss[k] for k in keys])
            if (i + 1) % self.log_step == 0:
                et = str(datetime.timedelta(seconds=time.time() - start_time))[:-7]
                log = "Elapsed [{}], Iteration [{}/{}]".format(et, i + 1, self.num_iters)
                for tag in keys:
                    log += ", {}: {:.4f}".format(tag, loss[tag])
                print(log)
        return history


class GANSolver(Solver):
    """Mirror of train_with_discriminator.py:Solver (train_with_discriminator.py:13-145): the
    generator step of train.py plus Discriminator() on the real and the reconstructed mel,
    d_loss = BCE(D(x_real), 1) + BCE(D(x_psnt), 0) added to the generator loss, ONE backward,
    then g_optimizer.step() and d_optimizer.step() (:102-111) -- the discriminator minimises
    the same loss the generator does, as in the reference.  wandb logging (:126-134) is
    replaced by the same line printed to stdout."""

    def build_model(self):
        from .factory.Discriminator import Discriminator

        super().build_model()
        self.G = self.VC
        self.g_optimizer = self.vc_optimizer
        self.D = Discriminator().to(self.device)
        _, dflat, dgflat = D.flatten_params_(self.D)
        self.d_optimizer = FusedAdam(dflat, dgflat, 0.0001)

    def reset_grad(self):
        self.g_optimizer.zero_grad()
        self.d_optimizer.zero_grad()

    def discriminator_loss(self, real, fake):
        return discriminator_loss(real, fake)

    def train(self):
        keys = ["G/loss_id", "G/loss_id_psnt", "G/loss_cd", "D/loss_d"]
        print("Start training...")
        start_time = time.time()
        data_iter = None
        history = []
        for i in range(self.num_iters):
            try:
                x_real, emb_org = next(data_iter)
            except Exception:
                data_iter = iter(self.vcc_loader)
                x_real, emb_org = next(data_iter)
            x_real = x_real.to(self.device)
            emb_org = emb_org.to(self.device)
            self.G = self.G.train()
            g_loss, (l_id, l_id_psnt, l_cd), x_psnt = vc_losses(self.G, x_real, emb_org, self.lambda_cd)
            d_loss = self.discriminator_loss(self.D(x_real), self.D(x_psnt.squeeze()))
            g_loss = g_loss + d_loss
            self.reset_grad()
            g_loss.backward()
            join_side()
            self.g_optimizer.step()
            self.d_optimizer.step()
            loss = self._read(keys, (l_id, l_id_psnt, l_cd, d_loss))
            history.append([loss[k] for k in keys])
            if (i + 1) % self.log_step == 0:
                et = str(datetime.timedelta(seconds=time.time() - start_time))[:-7]
                log = "Elapsed [{}], Iteration [{}/{}]".format(et, i + 1, self.num_iters)
                for tag in keys:
                    log += ", {}: {:.4f}".format(tag, loss[tag])
                print(log)
        return history


# ------------------------------------------------------------------------- command line (C1 driver)
class Config:
    """The reference's Config (train.py:134-150) plus the build's shape / precision flags."""

    def __init__(self, model_name, data_dir, device, num_iters, isadain, batch_size=2, len_crop=176, freq=22,
                 log_step=10):
        self.model_name = model_name
        self.data_dir = data_dir
        self.num_iters = num_iters
        self.isadain = isadain
        self.device = device
        self.batch_size = batch_size
        self.len_crop = len_crop
        self.lambda_cd = 1
        self.lambda_ad = 1
        self.dim_neck = 44
        self.dim_emb = 256
        self.dim_pre = 512
        self.freq = freq
        self.log_step = log_step


class SyntheticUtterances:
    """Endless synthetic batches of the metric's shape: batch i is
    detinit.det_inputs(batch_size, len_crop, seed=seed + i) -- log10-mel-like values in [-5, 2]
    and unit-norm 256-d speaker embeddings -- as CPU tensors, the form get_loader yields."""

    def __init__(self, batch_size, len_crop, dim_emb=256, seed=1234):
        self.batch_size, self.len_crop, self.dim_emb, self.seed = batch_size, len_crop, dim_emb, seed

    def __iter__(self):
        from .detinit import det_inputs

        i = 0
        while True:
            x, e = det_inputs(self.batch_size, self.len_crop, self.dim_emb, seed=self.seed + i)
            yield torch.from_numpy(x), torch.from_numpy(e)
            i += 1


def build_parser():
    import argparse

    p = argparse.ArgumentParser(
        prog="python -m autoformer_amd.train",
        description="AutoVC-family training on the MI355X: train.py (Solver), train_with_discriminator.py "
                    "(--discriminator) and train_with_adjust.py (the *_Adjust models) over the HIP kernels.")
    # the reference's flags (train.py:152-159)
    p.add_argument("--model_name", default="AutoVC", help="traning model name (a factory plugin)")
    p.add_argument("--data_dir", help="traning data folder (train.pkl + mel .npy files)")
    p.add_argument("--save_model_name")
    p.add_argument("--use_adain", default=False)
    p.add_argument("--device", default="cuda:0")
    p.add_argument("--num_iters", default=1000000, help="iter time")
    # the build's flags (BASELINE C1)
    p.add_argument("--batch_size", type=int, default=2)
    p.add_argument("--len_crop", type=int, default=176)
    p.add_argument("--freq", type=int, default=22)
    p.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32",
                   help="compute precision of the HIP kernels (fp32: the reference's arithmetic)")
    p.add_argument("--synthetic", action="store_true", help="synthetic batches instead of --data_dir")
    p.add_argument("--seed", type=int, default=1234, help="first synthetic batch seed")
    p.add_argument("--det_init", action="store_true",
                   help="closed-form weights (autoformer_amd.detinit, the goldens' initialiser)")
    p.add_argument("--discriminator", action="store_true", help="train_with_discriminator.py's two-model step")
    p.add_argument("--log_step", type=int, default=10)
    return p


def main(argv=None):
    """Parse, build the reference's Solver for the flags and train; returns the per-iteration losses."""
    args = build_parser().parse_args(argv)
    import autoformer_amd as A

    if not args.synthetic and not args.data_dir:
        raise SystemExit("one of --data_dir or --synthetic is required")
    if not str(args.device).startswith("cuda"):
        raise SystemExit(f"--device {args.device}: the HIP kernels need a GPU (the CPU counterpart is the "
                         "oracle, oracle/autovc_cpu.py OracleSolver, test infrastructure only)")
    A.set_compute(args.dtype)
    config = Config(args.model_name, args.data_dir, args.device, int(args.num_iters), bool(args.use_adain),
                    args.batch_size, args.len_crop, args.freq, args.log_step)
    if args.synthetic:
        loader = SyntheticUtterances(args.batch_size, args.len_crop, config.dim_emb, args.seed)
    else:
        from .data import get_loader

        loader = get_loader(args.data_dir, dim_neck=config.dim_neck, batch_size=args.batch_size,
                            len_crop=args.len_crop)
    if args.model_name.endswith("_Adjust"):
        cls = AdjustSolver
    elif args.discriminator:
        cls = GANSolver
    else:
        cls = Solver
    solver = cls(loader, config)
    if args.det_init:
        from .detinit import det_init_

        for m in [solver.VC] + ([solver.D] if args.discriminator else []):
            det_init_(m)
    history = solver.train()
    if args.save_model_name:
        torch.save(solver.VC.state_dict(), f"{args.save_model_name}.pt")
    return history


if __name__ == "__main__":
    main()
