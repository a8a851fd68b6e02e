"""Full-size op-level parity of the kernels bench.py times.

One production TrainStep step (bf16 compute, gradient sink on, the persistent / wavefront
recurrences, split-K weight gradients, halo convolutions, fused BN epilogues, the lstm1 fold)
at BASELINE.json's configurations, with every GEMM, LSTM recurrence, BN pass and code expansion
intercepted (tests/capture_ref.py): each op's outputs are checked against a float64
computation on the SAME inputs the kernel read, at OP_BAR relative Frobenius.  This holds the
timed kernels themselves to a tight bar at full size; the fp32 golden tests (1e-3) keep pinning
the math to the reference at small batch.

  C2: AutoVC B=64 T=128 freq=16 (reference factory/AutoVC.py:26-41,96,110)
  C4: MetaConv B=64 T=176 freq=22 (reference factory/MetaConv.py:23-76, MLPMixer.py:16-33,58-92,
      Norm.py:53-60: GroupNorm, LayerNorm, GELU twins, patchify, batched transposes)
  MetaPool B=64 T=176 (factory/MetaPool.py:7-77: the pooling mixer)
  C5: AutoVC + Discriminator B=64 T=176 (train_with_discriminator.py:90-111,
      factory/Discriminator.py:18-29: the dense head, BCE)
Every config also holds the loss block (train.py:84-96) and the fused Adam (train.py:99).
"""
import importlib

import pytest
import torch

from tests.capture_ref import Capture

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
OP_BAR = 1e-2
STEP_OPS = ["vc_loss", "vc_loss_grad", "adam"]  # the loss block and the optimizer of every step


def _synthetic(B, T, seed=0):
    g = torch.Generator().manual_seed(1234 + seed)
    x = torch.clamp(torch.randn(B, T, 80, generator=g) * 1.5 - 2.5, -5.0, 2.0)
    g2 = torch.Generator().manual_seed(5678 + seed)
    e = torch.nn.functional.normalize(torch.randn(B, 256, generator=g2), dim=-1)
    return x.to(DEV), e.to(DEV)


def _run(name, freq, B, T, disc=False):
    import autoformer_amd as A
    from autoformer_amd.detinit import det_init_
    from autoformer_amd.layers import set_grad_sink
    from autoformer_amd.train import TrainStep

    A.set_compute("bf16")
    cls = getattr(importlib.import_module(f"autoformer_amd.factory.{name}"), name)
    m = cls(44, 256, 512, freq)
    det_init_(m)
    m = m.to(DEV).train()
    x, e = _synthetic(B, T)
    Dm, extra = None, None
    if disc:
        from autoformer_amd.factory.Discriminator import Discriminator
        from autoformer_amd.train import gan_extra

        Dm = Discriminator(crop_len=T)
        det_init_(Dm)
        Dm = Dm.to(DEV).train()
        extra = gan_extra(Dm)
    ts = TrainStep(m, lr=1e-4, extra=extra, extra_modules=[Dm] if disc else ())
    try:
        ts.step(x, e)  # warm: packs built, workspaces allocated
        torch.cuda.synchronize()
        with Capture() as cap:
            ts.step(x, e)
            torch.cuda.synchronize()
        ts.check()
    finally:
        set_grad_sink(False)
    print(f"\n{name}{'+D' if disc else ''} B={B} T={T}: " + cap.summary(20))
    return cap


def _assert(cap, must):
    ops = {op for op, _, _ in cap.records}
    missing = set(must) - ops
    assert not missing, f"ops not exercised: {missing}"
    bad = [(v, tag, k) for v, op, tag, k in cap.worst() if not v <= OP_BAR]
    assert not bad, bad[:10]


@pytest.mark.timeout(600)
def test_c2_ops_vs_fp64():
    cap = _run("AutoVC", 16, 64, 128)
    _assert(cap, ["gemm", "lstm_fwd", "lstm2_fwd", "lstm_bwd", "lstm2_bwd", "lstm_fwd_fold", "lstm_bwd_fold",
                  "code_cat", "bn_apply", "bn_bwd", "conv_edge_table", "conv_edge_colsum"] + STEP_OPS)
    tags = " | ".join(t for _, t, _ in cap.records)
    # the decoder lstm2 backward runs as the two-layer wavefront launch, lstm1's as the folded single-layer one
    assert "lstm2_bwd B64 T128 H1024" in tags and "lstm_bwd_fold B64 T128 H512 nc8" in tags
    assert " sk" in tags and " win" in tags and " acc" in tags and " rowbias" in tags


@pytest.mark.timeout(600)
def test_c4_ops_vs_fp64():
    cap = _run("MetaConv", 22, 64, 176)
    _assert(cap, ["gemm", "bn_apply", "bn_bwd", "group_norm_fwd", "group_norm_bwd", "layer_norm_fwd",
                  "layer_norm_bwd", "patchify", "btranspose"] + STEP_OPS)
    tags = " | ".join(t for _, t, _ in cap.records)
    assert " gelu" in tags and " dgelu" in tags  # the GELU forward / backward epilogues of the mixer
    assert " colsum" in tags  # the mixer's bias gradients in the dgelu epilogue


@pytest.mark.timeout(600)
def test_metapool_ops_vs_fp64():
    cap = _run("MetaPool", 22, 64, 176)
    _assert(cap, ["gemm", "pool3", "group_norm_fwd", "group_norm_bwd", "layer_norm_fwd"] + STEP_OPS)
    tags = " | ".join(t for _, t, _ in cap.records)
    assert "pool3 B64 L176" in tags and " bwd" in tags


@pytest.mark.timeout(600)
def test_c5_ops_vs_fp64():
    cap = _run("AutoVC", 22, 64, 176, disc=True)
    _assert(cap, ["gemm", "lstm_fwd", "lstm2_fwd", "lstm_bwd", "lstm2_bwd", "bn_apply", "bn_bwd", "disc_dense_fwd",
                  "disc_dense_bwd", "bce_loss", "bce_grad"] + STEP_OPS)
