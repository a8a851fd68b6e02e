#!/usr/bin/env python
"""Benchmark: mel-frames/s of the AutoVC train.py step (fwd + encoder re-pass + MSE/L1 +
bwd + Adam) on synthetic (B, T, 80) batches resident in HBM, 1..N GPUs (one process per
GPU, data parallel, RCCL gradient all-reduce).

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

With --gpus N > 1 and no launcher environment (WORLD_SIZE unset) the script starts the N
ranks itself: N child processes of this script with RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR=127.0.0.1 / MASTER_PORT set, started before this process touches the GPU.  Every
rank checks that the process group it joined has exactly N ranks.

Prints ONE JSON line on rank 0 (see DESIGN.md §Measurement for every field).
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "mel-frames/sec fwd+bwd, AutoVC 80×128 mel, batch=64, at 1/2/4/8 GPUs"
PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_F32_TFLOPS = 157.3     # f32 MFMA
# dense bf16 MFMA peak measured on the box: 16x16x32 chains on every CU, 2.05 GHz under that load
# (tools/probes/mfma_peak.hip, profiles/r6_mfma_peak.txt)
PEAK_BF16_MEASURED_TFLOPS = 2047.4
# algorithmic work of one train step per mel frame (torch flop counter on the reference)
FLOP_PER_FRAME = {("AutoVC", 128, 16): 191.55e6, ("AutoVC", 176, 22): 191.59e6, ("AutoVC+D", 176, 22): 191.87e6,
                  ("MetaConv", 176, 22): 1044.41e6, ("MetaPool", 176, 22): 981.86e6,
                  # model variants, same counter: tools/variant_flops.py
                  ("AutoVC2", 128, 16): 194.93e6, ("AutoVC2", 176, 22): 194.98e6,
                  ("AutoVC_Adjust", 128, 16): 492.84e6, ("AutoVC_Adjust", 176, 22): 492.97e6,
                  ("MetaConv2", 176, 22): 1047.80e6, ("MetaPool2", 176, 22): 985.24e6,
                  ("MetaConv_Adjust", 176, 22): 1345.79e6, ("MetaPool_Adjust", 176, 22): 1081.17e6}
VARIANTS = ["AutoVC2", "AutoVC_Adjust", "MetaConv2", "MetaPool2", "MetaConv_Adjust", "MetaPool_Adjust"]


def synthetic_batch(B, T, rank, device):
    """log10-mel-like clamp(N(-2.5, 1.5^2), -5, 2), unit-norm embeddings."""
    g = torch.Generator().manual_seed(1234 + rank)
    x = torch.clamp(torch.randn(B, T, 80, generator=g) * 1.5 - 2.5, -5.0, 2.0)
    g2 = torch.Generator().manual_seed(5678 + rank)
    e = torch.nn.functional.normalize(torch.randn(B, 256, generator=g2), dim=-1)
    return x.to(device), e.to(device)


DOMINANT = "lstm_persist_bwd<1024>"
DOMINANT_WAVE = "lstm2_persist_bwd<1024>"
PEAK_HBM_GBS = 8000.0       # MI355X HBM3E (MI355X_MICROARCH.md)


def wavefront_bwd(B):
    """Whether the step runs the decoder lstm2 backward as the two-layer wavefront launch."""
    from autoformer_amd import kernels as K
    from autoformer_amd import layers as Ly

    return Ly._PAIR_BWD and K.lstm2_bwd_persistent(B, 1024)


def kernel_timing_wave(model, B, T, reps=3):
    """Isolated replays of lstm2_persist_bwd<1024> (the decoder lstm2 backward, BOTH layers in one
    wavefront launch of T + 1 ticks): the dominant kernel when the step runs it.  FLOP per launch: the
    three recurrent products per step (W_hh1^T, W_ih1^T, W_hh0^T: 2 * B * 4H * H each) over T steps.
    Algorithmic bytes: the three transposed weights once (3 * 4H * H bf16) + per step
    dL/dh1 fp32 (B*H*4) + per layer c_t, c_{t-1} fp32 (2*B*H*4) + gates fp32 (B*4H*4) + dG out: bf16
    (B*4H*2) in the step's form (bf16 dG + per-group bias partials, ABI 28); timed in that form."""
    from autoformer_amd import kernels as K
    from autoformer_amd import layers as Ly

    c0, c1 = model.decoder._lstm2
    wt0 = c0.packs()[3]
    _, _, _, wt1, wti1 = c1.packs()
    H = c0.H
    dev = wt0.device
    g = torch.Generator(device=dev).manual_seed(7)
    dh = torch.randn(B * T, H, device=dev, generator=g) * 0.1
    cs = [torch.randn(B * T, H, device=dev, generator=g) * 0.5 for _ in range(2)]
    gs = [torch.rand(B * T, 4 * H, device=dev, generator=g) for _ in range(2)]
    db = True  # the step's form (layers._LSTMPairFn.backward)
    K.lstm2_bwd(dh, cs[0], gs[0], cs[1], gs[1], wt0, wti1, wt1, B, T, H, fp32=not db, db=db)  # warm
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        K.lstm2_bwd(dh, cs[0], gs[0], cs[1], gs[1], wt0, wti1, wt1, B, T, H, fp32=not db, db=db)
    e1.record(s)
    torch.cuda.synchronize()
    K.check_faults()
    avg_us = e0.elapsed_time(e1) * 1e3 / reps
    G = 4 * H
    alg_bytes = 3 * G * H * 2 + T * (B * H * 4 + 2 * (2 * B * H * 4 + B * G * 4 + B * G * (2 if db else 6)))
    return {"kernel": DOMINANT_WAVE + " (decoder lstm2 backward, both layers in one wavefront launch, T=%d, B=%d, "
            "H=%d)" % (T, B, H), "avg_us": avg_us, "bytes": float(alg_bytes), "flops": 3 * 2.0 * B * G * H * T}


def kernel_timing(model, B, T, reps=3):
    """Isolated replays of the dominant kernel (HIP events on its launch stream): the secondary
    `avg_us_isolated` figure.  The roofline's `avg_us` is the mean over the launches inside the
    timed region (kernels.LAUNCH_TIMING), where the side-stream GEMMs share the chip with it.

    The kernel is lstm_persist_bwd<1024>: the whole backward recurrence of one decoder lstm2
    layer (H=1024, B=64, T steps) in one launch, the largest single-kernel share of the step
    (profiles/).  Algorithmic bytes per launch: W_hh^T once (4H*H bf16) + per
    step dh, c fp32 (2*B*H*4) + activated gates fp32 (B*4H*4) + dG fp32 and bf16 out (B*4H*6)."""
    from autoformer_amd import kernels as K

    core = model.decoder._lstm2[1]
    whh, whh_t = core.packs()[2:4]
    H = core.H
    dev = whh.device
    g = torch.Generator(device=dev).manual_seed(7)
    dh = torch.randn(B * T, H, device=dev, generator=g) * 0.1
    h = torch.randn(B * T, H, device=dev, generator=g) * 0.5
    c = torch.randn(B * T, H, device=dev, generator=g) * 0.5
    gates = torch.rand(B * T, 4 * H, device=dev, generator=g)
    if not K.lstm_persistent_bwd(B, H, 1):
        raise RuntimeError("bench: the persistent backward recurrence does not apply to this shape/device")
    gbuf = K.lstm_bwd_scratch(B, H, 1, dev)
    K.lstm_bwd(dh, h, c, gates, whh, whh_t, B, T, H, 1, gbuf=gbuf)  # warm
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        K.lstm_bwd(dh, h, c, gates, whh, whh_t, B, T, H, 1, gbuf=gbuf)
    e1.record(s)
    torch.cuda.synchronize()
    if K.lstm_bwd_timeout_flag(gbuf, B, H):
        raise RuntimeError("bench: persistent LSTM backward hit its spin timeout")
    avg_us = e0.elapsed_time(e1) * 1e3 / reps
    G = 4 * H
    alg_bytes = G * H * 2 + T * (2 * B * H * 4 + B * G * 4 + B * G * 6)
    return {"kernel": DOMINANT + " (decoder lstm2 backward recurrence, one launch = T=%d steps, B=%d, H=%d)"
            % (T, B, H), "avg_us": avg_us, "bytes": float(alg_bytes), "flops": 2.0 * B * G * H * T}


def _names(kernel, name):
    """Whether a profiler kernel name is `kernel` ("f<1024>") with any further template
    arguments ("f<1024, false>"), and not another kernel sharing its prefix ("f_ps<1024>")."""
    base, args = kernel.rstrip(">").split("<")
    return f"{base}<{args}>" in name or f"{base}<{args}," in name


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/r*_pmc_traffic.json, written by tools/rocpd_summary.py from separate
    FETCH_SIZE / WRITE_SIZE rocprofv3 passes, FETCH_SIZE doubled per MI355X_MICROARCH.md)."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")))
    if not files:
        return None, None
    data = json.load(open(files[-1]))["kernels"]
    for name, e in data.items():
        if _names(kernel, name) and "hbm_bytes_per_launch" in e:
            return e["hbm_bytes_per_launch"], os.path.relpath(files[-1], ROOT)
    return None, None


def host_cores():
    """(physical cores of the host, CPUs this process may run on)."""
    phys = set()
    try:
        cur = {}
        for line in open("/proc/cpuinfo"):
            if ":" not in line:
                if cur:
                    phys.add((cur.get("physical id"), cur.get("core id")))
                cur = {}
                continue
            k, v = (x.strip() for x in line.split(":", 1))
            cur[k] = v
        if cur:
            phys.add((cur.get("physical id"), cur.get("core id")))
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count()
    return len(phys) or None, aff


def pmc_mfma(kernel):
    """MFMA counters of `kernel` from the newest committed counter pass (profiles/r*_pmc_mfma_step.json,
    tools/gpu_pmc.sh + tools/pmc_mfma.py): bf16 MFMA TFLOP/s from SQ_INSTS_VALU_MFMA_MOPS_BF16 over the
    dispatch time, the fraction of wave cycles waiting (SQ_WAIT_ANY), and its source file."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_mfma_step.json")))
    if not files:
        return None
    data = json.load(open(files[-1]))
    for name, e in data.items():
        if _names(kernel, name):
            return {"mfma_instr_tflops": round(e.get("bf16_tflops", 0.0), 1),
                    "mfma_instr_frac": round(e.get("bf16_tflops", 0.0) / PEAK_BF16_TFLOPS, 4),
                    "wave_wait_frac": round(e.get("wait", 0.0), 3), "source": os.path.relpath(files[-1], ROOT),
                    "note": "MFMA instruction rate (lstm_persist_bwd: 16-row tiles with 8 utterances, 2x the useful "
                            "FLOPs; lstm2_persist_bwd: full 16-utterance tiles)"}
    return None


def cpu_baseline(B, T, freq, steps=5):
    """The CPU oracle (oracle/autovc_cpu.py, the pinned restatement of the reference) timed on
    this box's host cores: same step, fp32, bounded sample of 1 warm-up + `steps` steps, the
    MEDIAN step reported.  `cores` = the intra-op threads torch ran the oracle
    with: the CPU share the GPU pool grants one GPU's process (OMP_NUM_THREADS, 16 on the box),
    not the host's physical core count (128) -- that many threads would run on CPUs other jobs of
    the host own."""
    from oracle import autovc_cpu as O

    x, e = synthetic_batch(B, T, 0, "cpu")
    s = O.OracleSolver(freq=freq)
    s.step(x, e)
    times = []
    for _ in range(steps):
        t0 = time.perf_counter()
        s.step(x, e)
        times.append(time.perf_counter() - t0)
    dt = sorted(times)[len(times) // 2]
    phys, aff = host_cores()
    return {"value": round(B * T / dt, 1), "unit": "mel-frames/s", "cores": torch.get_num_threads(),
            "kind": "port", "host_physical_cores": phys, "host_cpus_allowed": aff,
            "cores_note": "intra-op threads = the per-GPU CPU share of the pool (OMP_NUM_THREADS), not the host's "
                          "physical cores",
            "sample": f"oracle train step B={B} T={T} freq={freq} fp32, 1 warm-up + {steps} timed steps, median "
                      f"{dt * 1e3:.0f} ms/step (min {min(times) * 1e3:.0f}, max {max(times) * 1e3:.0f}), "
                      f"{torch.get_num_threads()} intra-op threads"}


def launch_ranks(n):
    """Start n ranks of this script (one per GPU) and wait for them; returns the exit code.
    The parent never touches the GPU (torch.cuda.device_count() does not initialise HIP on
    this image), so no process that initialised the GPU forks or execs."""
    import socket
    import subprocess

    have = torch.cuda.device_count()
    if have < n:
        print(f"bench.py: --gpus {n} needs {n} visible GPUs, this node has {have}", file=sys.stderr, flush=True)
        return 2
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                c = p.poll()
                if c is None:
                    continue
                pending.remove(p)
                if c != 0 and rc == 0:
                    rc = c
                    for q in pending:  # one rank failed: the others would wait on it forever
                        q.terminate()
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--len-crop", type=int, default=None, help="default 128 (AutoVC), 176 (MetaConv/MetaPool/--disc)")
    ap.add_argument("--freq", type=int, default=None, help="default 16 at T=128, 22 at T=176")
    ap.add_argument("--model", default="AutoVC", choices=["AutoVC", "MetaConv", "MetaPool"] + VARIANTS,
                    help="factory plugin (train.py / train_with_adjust.py --model_name); the MetaFormer "
                         "families hard-wire T=176")
    ap.add_argument("--disc", action="store_true",
                    help="AutoVC + Discriminator two-model step (train_with_discriminator.py), T=176")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--replay", action="store_true",
                    help="record one step's native calls and replay them (autoformer_amd/replay.py): the eager "
                         "step's kernels, streams and event edges without its Python -- the default")
    ap.add_argument("--eager", action="store_true",
                    help="step from Python every time (no recorded replay)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    # diagnostic ablations skip work inside the step: a number measured under them is not the metric
    skipped = [k for k in ("AVC_ABLATE_WGRAD",) if os.environ.get(k, "0") not in ("", "0")]
    if skipped:
        raise SystemExit(f"bench.py: diagnostic ablation(s) {skipped} set; they skip work in the timed step")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))

    import importlib

    from autoformer_amd import dist as D
    from autoformer_amd import set_compute
    from autoformer_amd.detinit import det_init_
    from autoformer_amd.train import TrainStep, gan_extra

    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    if env_world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the process group has {env_world} rank(s) "
                         f"(WORLD_SIZE={os.environ.get('WORLD_SIZE')})")
    if args.gpus > 1:
        # RCCL binds the communicator to the current device when the group is created
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    rank, world, local = D.init_from_env("nccl")
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the process group has {world} rank(s) "
                         f"(WORLD_SIZE={os.environ.get('WORLD_SIZE')})")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    set_compute(args.dtype)
    if args.disc and args.model != "AutoVC":
        raise SystemExit("--disc pairs the Discriminator with AutoVC (train_with_discriminator.py)")
    wide = args.model.startswith("Meta") or args.disc
    B = args.batch
    T = args.len_crop if args.len_crop is not None else (176 if wide else 128)
    freq = args.freq if args.freq is not None else (22 if T == 176 else 16)
    name = "AutoVC+D" if args.disc else args.model

    # the reference's plugin lookup (train.py:45-47)
    cls = getattr(importlib.import_module(f"autoformer_amd.factory.{args.model}"), args.model)
    model = cls(44, 256, 512, freq)
    det_init_(model)
    model = model.to(dev).train()
    x, e = synthetic_batch(B, T, rank, dev)
    if args.disc:
        from autoformer_amd.factory.Discriminator import Discriminator

        disc = Discriminator(crop_len=T)
        det_init_(disc)
        disc = disc.to(dev).train()
        trainer = TrainStep(model, lr=1e-4, extra=gan_extra(disc), extra_modules=[disc])
    else:
        trainer = TrainStep(model, lr=1e-4)

    # the recorded replay (replay.py) is the default step form of the AutoVC steps: the same kernels,
    # streams and event edges as the eager step, with no per-kernel Python, so a slow host does not
    # set the step time.  The MetaConv / MetaPool steps (~29 ms) are never host-bound and ran ~1 %
    # faster eager (29.13-29.23 vs 29.52-29.54 ms, profiles/r5_replay_ab.txt): eager unless --replay
    host_bound = args.model not in ("MetaConv", "MetaPool")
    replay = not args.eager and (args.replay or host_bound)
    for _ in range(args.warmup):
        trainer.step(x, e)
    if replay:
        trainer.record(x, e, warmup=0)
        trainer.step(x, e)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    from autoformer_amd import kernels as K

    # dominant-kernel launches inside the timed region, timed by HIP events on their stream
    K.LAUNCH_TIMING = [] if (not args.no_kernel_timing and args.model == "AutoVC") else None
    if world > 1:
        trainer.comm_timing = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = trainer.step(x, e)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    comm_ms = 0.0
    if world > 1:
        comm_ms = sum(a.elapsed_time(b) for a, b in trainer.comm_timing) / args.steps
        trainer.comm_timing = None
        t = torch.tensor([elapsed, comm_ms], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, comm_ms = t[0].item(), t[1].item()
    trainer.check()  # a persistent recurrence that timed out invalidates the run: raise
    loss_v = float(loss.item())
    ms = elapsed / args.steps * 1e3
    frames = world * B * T
    value = frames / (elapsed / args.steps)

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    fpf = FLOP_PER_FRAME.get((name, T, freq))
    peak = PEAK_BF16_TFLOPS if args.dtype == "bf16" else PEAK_F32_TFLOPS
    step = ("train_with_discriminator.py step (G fwd + encoder re-pass + D on real/fake + 2xMSE + L1 + 2xBCE + "
            "one bwd + both Adams)" if args.disc else
            "train_with_adjust.py step (fwd with 2 Adjust passes + encoder re-pass with 1 + 2xMSE + 2xL1 + bwd + "
            "Adam)" if args.model.endswith("_Adjust") else
            "train.py step (fwd + encoder re-pass + 2xMSE + L1 + bwd + Adam)")
    default = name == "AutoVC" and (T, freq) == (128, 16)
    metric = METRIC if default else f"mel-frames/sec fwd+bwd, {name} 80\u00d7{T} mel, batch={B}"
    out = {"metric": metric, "value": round(value, 1), "unit": "mel-frames/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": args.dtype, "data": "synthetic",
           "config": {"workload": f"{name} {step}, B={B}/GPU, T={T}, freq={freq}, dim_neck=44, dim_emb=256, "
                                  f"dim_pre=512",
                      "global_batch": B * world, "seq_len": T, "freq": freq, "parallelism": f"dp{world}",
                      "launch": "replay" if replay else "eager"},
           "step_mfma_frac": round(value * fpf / (world * peak * 1e12), 5) if fpf else None,
           "final_loss": loss_v}
    if world > 1:
        # main-stream time per step spent waiting for the gradient average after the backward
        # (the decoder / postnet slice overlaps the encoder backward), max over ranks
        out["allreduce_ms"] = round(comm_ms, 4)
        out["allreduce_bytes_per_step"] = trainer.gflat.numel() * trainer.gflat.element_size()
        out["collective"] = f"{dist.get_backend()} all_reduce AVG, {D.BUCKET_BYTES >> 20} MiB buckets"
    if not args.no_kernel_timing and args.model == "AutoVC":
        evs, K.LAUNCH_TIMING = K.LAUNCH_TIMING or [], None
        wave = wavefront_bwd(B)
        dominant = DOMINANT_WAVE if wave else DOMINANT
        # isolated replays (also: algorithmic bytes / FLOP)
        kt = kernel_timing_wave(model, B, T) if wave else kernel_timing(model, B, T)
        if evs:  # the in-step launches of the timed region (beside the side-stream GEMMs)
            step_us = sum(a.elapsed_time(b) for a, b in evs) * 1e3 / len(evs)
        else:
            step_us = kt["avg_us"]
        # the path's roofline is dense bf16 MFMA; HBM is the secondary counter
        tfs = kt["flops"] / (step_us * 1e-6) / 1e12
        gbs = kt["bytes"] / (step_us * 1e-6) / 1e9
        traffic, src = pmc_traffic(dominant)
        out["roofline"] = {"bound": "mfma", "achieved": round(tfs, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                           "frac": round(tfs / PEAK_BF16_TFLOPS, 5),
                           "peak_measured": PEAK_BF16_MEASURED_TFLOPS,
                           "frac_measured": round(tfs / PEAK_BF16_MEASURED_TFLOPS, 5),
                           "peak_measured_source": "profiles/r6_mfma_peak.txt",
                           "traffic": traffic, "kernel": kt["kernel"],
                           "avg_us": round(step_us, 3), "launches_timed": len(evs),
                           "avg_us_isolated": round(kt["avg_us"], 3), "flop_per_launch": kt["flops"],
                           "alg_bytes_per_launch": kt["bytes"], "hbm_achieved_gbs": round(gbs, 1),
                           "hbm_frac": round(gbs / PEAK_HBM_GBS, 5), "traffic_source": src,
                           "counters": pmc_mfma(dominant)}
    if world == 1 and not args.no_cpu_baseline and default:
        out["cpu_baseline"] = cpu_baseline(B, T, freq)
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
