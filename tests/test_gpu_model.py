"""Whole-model parity on the MI355X: the HIP AutoVC against the reference goldens
(tests/golden, generated from /root/reference) and the CPU oracle.

Bars: fp32 mel_postnet rel-inf <= 1e-3 (north star); losses rel <= 1e-4;
grads rel-Frobenius <= 1e-2 per tensor with an absolute floor of 1e-6 for the conv biases
that feed a BatchNorm (analytically zero gradient); bf16 mode loose (rel-inf <= 5e-2).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F


pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def rel_inf(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)


def _model(freq, comp="fp32"):
    import autoformer_amd as A
    from autoformer_amd.detinit import det_init_
    from factory.AutoVC import AutoVC

    A.set_compute(comp)
    m = AutoVC(44, 256, 512, freq)
    det_init_(m)
    return m.to(DEV).train()


def _step(m, x, e):
    x_id, x_psnt, code = m(x, e, e)
    l1 = F.mse_loss(x, x_id.squeeze())
    l2 = F.mse_loss(x, x_psnt.squeeze())
    code_re = m(x_psnt, e, None)
    l3 = F.l1_loss(code, code_re)
    return (x_id, x_psnt, code, code_re), (l1, l2, l3), l1 + l2 + l3


@pytest.mark.parametrize("fname", ["autovc_T176.npz", "autovc_T128.npz"])
def test_autovc_fp32_matches_reference_goldens(golden, fname):
    g = golden(fname)
    m = _model(int(g["freq"]))
    x, e = torch.from_numpy(g["x"]).to(DEV), torch.from_numpy(g["emb"]).to(DEV)
    outs, losses, total = _step(m, x, e)
    m.zero_grad()
    total.backward()
    torch.cuda.synchronize()
    assert rel_inf(outs[1].detach().cpu(), g["mel_psnt"]) < 1e-3
    assert rel_inf(outs[0].detach().cpu(), g["mel"]) < 1e-3
    assert rel_inf(outs[2].detach().cpu(), g["codes"]) < 1e-3
    assert rel_inf(outs[3].detach().cpu(), g["codes_re"]) < 1e-3
    np.testing.assert_allclose([l.item() for l in losses], g["losses"], rtol=1e-4)
    bad = {}
    for name, p in m.named_parameters():
        ref_n = float(g["gnorm/" + name])
        got = p.grad.detach().cpu().double()
        head = g["ghead/" + name].astype(np.float64)
        err = np.abs(got.reshape(-1)[:64].numpy() - head).max()
        if "conv.bias" in name and "postnet.convolutions.4" not in name:
            ok = err < 1e-6 + 1e-2 * np.abs(head).max()
        else:
            # head bar: 1% of the larger of the head's max and the tensor's rms.  Any fp32
            # reordering of the forward (here the lstm1 fold: 1e-6 rel) can flip an isolated
            # ReLU unit sitting within 1e-7 of zero (measured: 1 of 131072 in decoder conv 2 at
            # T=128, tools/relu_flips.py), which moves the 64-element head of a gradient whose
            # entries are far below its rms (encoder.lstm.weight_hh_l1_reverse: head max 8e-4,
            # rms 1.4e-3) by ~1e-5; the norm check below stays at 1%.
            rms = ref_n / np.sqrt(max(p.numel(), 1))
            ok = abs(got.norm().item() - ref_n) <= 1e-2 * ref_n + 1e-6 and \
                err <= 1e-2 * max(np.abs(head).max(), rms, 1e-6)
        if not ok:
            bad[name] = (got.norm().item(), ref_n, err)
    assert not bad, bad
    for k, v in m.state_dict().items():
        if "running_" in k or "num_batches" in k:
            np.testing.assert_allclose(v.detach().cpu().numpy(), g["bn/" + k], rtol=1e-4, atol=1e-6, err_msg=k)


@pytest.mark.parametrize("fname", ["autovc_T176.npz", "autovc_T128.npz"])
def test_autovc_three_adam_steps_match_reference_solver(golden, fname):
    """train.py Solver semantics (train.py:82-99) with torch.optim.Adam over the HIP model."""
    g = golden(fname)
    m = _model(int(g["freq"]))
    opt = torch.optim.Adam(m.parameters(), 1e-4)
    got = []
    for i in range(3):
        x = torch.from_numpy(g[f"adam_x{i}"]).to(DEV)
        e = torch.from_numpy(g[f"adam_e{i}"]).to(DEV)
        _, losses, total = _step(m, x, e)
        opt.zero_grad()
        total.backward()
        opt.step()
        got.append([l.item() for l in losses])
    np.testing.assert_allclose(np.array(got), g["adam_losses"], rtol=2e-3)


@pytest.mark.parametrize("fname", ["autovc_T128.npz", "autovc_T176.npz"])
def test_autovc_bf16_loose(golden, fname):
    """The bf16 production model against the reference's fp32 goldens (B=2), held to the SURVEY
    §8(c) bf16 bar of 5e-2 as a relative Frobenius norm, and in the max norm to twice the
    reference's own bf16 drift on these inputs (the oracle under bf16 autocast against fp32,
    tools/bf16_drift.py, profiles/r5_bf16_drift_oracle.txt: mel_psnt rel-inf 4.95e-2 at T=128,
    4.19e-2 at T=176, mel 1.88e-2 / 1.68e-2 -- at B=2 one element sets it).  Every production op is
    held to 1e-2 against fp64 on its own inputs by tests/test_gpu_capture.py."""
    g = golden(fname)
    m = _model(int(g["freq"]), "bf16")
    x, e = torch.from_numpy(g["x"]).to(DEV), torch.from_numpy(g["emb"]).to(DEV)
    outs, losses, total = _step(m, x, e)
    total.backward()
    torch.cuda.synchronize()
    got, ref = outs[1].detach().cpu().double().numpy().ravel(), g["mel_psnt"].astype(np.float64).ravel()
    assert np.linalg.norm(got - ref) / np.linalg.norm(ref) < 5e-2
    assert np.abs(got - ref).max() / np.abs(ref).max() < 1e-1
    mel = outs[0].detach().cpu().double().numpy().ravel()
    assert np.linalg.norm(mel - g["mel"].ravel()) / np.linalg.norm(g["mel"]) < 5e-2
    assert np.abs(mel - g["mel"].ravel()).max() / np.abs(g["mel"]).max() < 4e-2
    np.testing.assert_allclose([l.item() for l in losses], g["losses"], rtol=5e-2)
    for p in m.parameters():
        assert torch.isfinite(p.grad).all()


def test_autovc_vs_oracle_batch8():
    """Larger batch than the goldens, against the CPU oracle on identical weights/inputs."""
    from autoformer_amd.detinit import det_inputs
    from oracle import autovc_cpu as O

    B, T, freq = 8, 64, 16
    x, e = det_inputs(B, T, seed=9)
    xt, et = torch.from_numpy(x), torch.from_numpy(e)
    sd = O.make_state(O.autovc_spec())
    losses_ref, total_ref, outs_ref = O.step_losses(lambda a, b, c: O.autovc_forward(sd, a, b, c, freq=freq), xt, et)
    m = _model(freq)
    outs, losses, total = _step(m, xt.to(DEV), et.to(DEV))
    assert rel_inf(outs[1].detach().cpu(), outs_ref[1].detach()) < 1e-3
    np.testing.assert_allclose([l.item() for l in losses], [l.item() for l in losses_ref], rtol=1e-4)


def _rel_frob(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


# bf16 bars at the bench configuration (B=64, T=128, freq=16): the REFERENCE computation's own bf16
# drift x 1.5 -- the CPU oracle under bf16 autocast (recurrences with bf16 operands and fp32 state, as
# on the GPU) against the same oracle in fp32, on these inputs (tools/bf16_drift.py,
# profiles/r5_bf16_drift_oracle.txt: mel_psnt rel-Frobenius 1.85e-2 / rel-inf 2.31e-2, mel 9.1e-3 /
# 9.6e-3, losses 1.7e-4, worst parameter gradient 0.132 (encoder conv BN bias, as on the GPU: 0.138),
# analytically-zero gradients 6.4e-4 of the largest norm)
B64_BARS = {"mel_psnt_frob": 2.8e-2, "mel_psnt_inf": 3.5e-2, "mel_frob": 1.4e-2, "mel_inf": 1.5e-2, "loss_rtol": 3e-4,
            "grad_frob": 0.2, "zero_grad_abs": 1e-3}


@pytest.mark.timeout(900)
def test_autovc_bf16_b64_vs_oracle():
    """The bf16 production model at the bench batch (B=64, T=128: 8192 frames, so the max-norm
    error is an extreme over 655k mel values, not one element) against the CPU oracle's fp32
    step on identical weights and inputs: outputs in the relative Frobenius and max norms, the
    three losses, and every parameter gradient (relative Frobenius)."""
    from autoformer_amd.detinit import det_inputs
    from oracle import autovc_cpu as O

    B, T, freq = 64, 128, 16
    x, e = det_inputs(B, T, seed=21)
    xt, et = torch.from_numpy(x), torch.from_numpy(e)
    torch.set_num_threads(min(16, torch.get_num_threads()))
    sd = O.make_state(O.autovc_spec())
    losses_ref, total_ref, outs_ref = O.step_losses(lambda a, b, c: O.autovc_forward(sd, a, b, c, freq=freq), xt, et)
    total_ref.backward()
    m = _model(freq, "bf16")
    outs, losses, total = _step(m, xt.to(DEV), et.to(DEV))
    total.backward()
    torch.cuda.synchronize()
    got = {
        "mel_psnt_frob": _rel_frob(outs[1].detach().cpu(), outs_ref[1].detach()),
        "mel_psnt_inf": rel_inf(outs[1].detach().cpu(), outs_ref[1].detach()),
        "mel_frob": _rel_frob(outs[0].detach().cpu(), outs_ref[0].detach()),
        "mel_inf": rel_inf(outs[0].detach().cpu(), outs_ref[0].detach()),
        "loss_rtol": max(abs(a.item() - b.item()) / abs(b.item()) for a, b in zip(losses, losses_ref)),
    }
    gref = {k: v.grad for k, v in sd.items() if v.requires_grad and v.grad is not None}
    gmax = max(float(g.norm()) for g in gref.values())
    rels, zeros = [], []
    for name, p in m.named_parameters():
        if name in gref and p.grad is not None:
            if float(gref[name].norm()) < 1e-6 * gmax:
                # analytically zero (a conv bias feeding a training-mode BatchNorm): absolute, scaled
                # by the largest gradient norm of the step
                zeros.append((float(p.grad.norm()) / gmax, name))
            else:
                rels.append((_rel_frob(p.grad.detach().cpu(), gref[name]), name))
    assert len(rels) + len(zeros) >= 70, f"only {len(rels) + len(zeros)} parameter gradients matched the oracle's names"
    rels.sort(reverse=True)
    got["grad_frob"] = rels[0][0]
    got["zero_grad_abs"] = max(zeros)[0] if zeros else 0.0
    print("\nbf16 B=64 vs oracle: " + " ".join(f"{k} {v:.3e}" for k, v in got.items()) + f" | worst grads "
          + ", ".join(f"{nm} {r:.2e}" for r, nm in rels[:5]) + f" | {len(zeros)} analytically-zero grads")
    bad = {k: (v, B64_BARS[k]) for k, v in got.items() if not v < B64_BARS[k]}
    assert not bad, bad


def test_encoder_list_api_and_eval_mode(golden):
    g = golden("autovc_T176.npz")
    m = _model(22)
    x, e = torch.from_numpy(g["x"]).to(DEV), torch.from_numpy(g["emb"]).to(DEV)
    codes = m.encoder(x, e)
    assert isinstance(codes, list) and len(codes) == 8 and codes[0].shape == (2, 88)
    m.eval()
    with torch.no_grad():
        mel, psnt, c = m(x, e, e)
    assert torch.isfinite(psnt).all()


def test_trainstep_sink_graph_matches_plain_autograd(golden):
    """TrainStep (flat buffers, gradient sink + side stream, fused Adam)
    reproduces the reference Solver's 3-step losses in fp32 compute."""
    from autoformer_amd.train import TrainStep
    from autoformer_amd.layers import set_grad_sink

    g = golden("autovc_T176.npz")
    m = _model(int(g["freq"]))
    ts = TrainStep(m, lr=1e-4)
    try:
        got = []
        for i in range(3):
            x = torch.from_numpy(g[f"adam_x{i}"]).to(DEV)
            e = torch.from_numpy(g[f"adam_e{i}"]).to(DEV)
            ts.step(x, e)
            torch.cuda.synchronize()
        # losses of the reference Solver are recorded before each step's update; recompute ours
        # by re-running the three steps on a fresh model and reading the fused losses
    finally:
        set_grad_sink(False)
    m2 = _model(int(g["freq"]))
    ts2 = TrainStep(m2, lr=1e-4)
    try:
        from autoformer_amd.train import vc_losses
        for i in range(3):
            x = torch.from_numpy(g[f"adam_x{i}"]).to(DEV)
            e = torch.from_numpy(g[f"adam_e{i}"]).to(DEV)
            _, parts, _ = vc_losses(m2, x, e)
            got.append([p.item() for p in parts])
            ts2.step(x, e)
    finally:
        set_grad_sink(False)
    np.testing.assert_allclose(np.array(got), g["adam_losses"], rtol=2e-3)
    for (n, p), (_, p2) in zip(m.named_parameters(), m2.named_parameters()):
        assert torch.allclose(p, p2, rtol=1e-4, atol=1e-6), n


def test_trainstep_recorded_replay_equals_eager_lr0():
    """The recorded replay of the step (replay.py) equals the eager step.  The bf16 step is not
    bit-reproducible (split-K atomics reorder run to run, and Adam's first updates turn sign flips of
    tiny gradients into whole-lr moves: two EAGER runs differ by up to 3 lr after 3 steps), so the
    parameters are held fixed (lr = 0) and the third step's losses and per-tensor gradients are
    compared (rel-Frobenius 1e-2: bf16 run-to-run spread 1.3e-3 measured); a missing or stale
    kernel in the replay shows as an O(1) error."""
    from autoformer_amd.detinit import det_inputs
    from autoformer_amd.layers import set_grad_sink
    from autoformer_amd.train import TrainStep

    x, e = det_inputs(4, 64, seed=3)
    x, e = torch.from_numpy(x).to(DEV), torch.from_numpy(e).to(DEV)
    ma, mb = _model(16, "bf16"), _model(16, "bf16")
    ta, tb = TrainStep(ma, lr=0.0), TrainStep(mb, lr=0.0)
    try:
        for _ in range(3):
            la = ta.step(x, e)
        tb.step(x, e)
        tb.record(x, e, warmup=0)   # = step 2, recorded
        lb = tb.step(x, e)          # replay = step 3
        torch.cuda.synchronize()
        assert abs(la.item() - lb.item()) <= 1e-4 * abs(la.item())
        assert torch.equal(ta.flat, tb.flat)  # lr = 0: nothing moved
        for (n, pa), (_, pb) in zip(ma.named_parameters(), mb.named_parameters()):
            ga, gb = pa.grad.double(), pb.grad.double()
            assert (ga - gb).norm() <= 1e-2 * ga.norm() + 1e-6, n  # SURVEY 8(c) gradient bar
        for (n, ba), (_, bb) in zip(ma.named_buffers(), mb.named_buffers()):
            assert torch.allclose(ba.double(), bb.double(), rtol=1e-4, atol=1e-6), n
    finally:
        set_grad_sink(False)


def test_host_inputs_refused_before_any_kernel():
    """A CPU input to a device model raises at the model's entry (K.require_device) instead of
    reaching a kernel as a host pointer (which faults the GPU)."""
    import factory.AutoVC as AV
    import factory.Discriminator as D

    m = AV.AutoVC(44, 256, 512, 16).to(DEV)
    x, e = torch.zeros(2, 128, 80), torch.zeros(2, 256)
    with pytest.raises(RuntimeError, match="HIP device tensors"):
        m(x, e.to(DEV), e.to(DEV))
    with pytest.raises(RuntimeError, match="HIP device tensors"):
        m(x.to(DEV), e, e.to(DEV))
    with pytest.raises(RuntimeError, match="HIP device tensors"):
        D.Discriminator().to(DEV)(x)
    torch.cuda.synchronize()
