"""The bf16 drift of the REFERENCE computation itself at the bench configuration (B=64, T=128,
freq=16): the CPU oracle step under torch.autocast(bfloat16) against the same oracle in fp32, on
the inputs and weights tests/test_gpu_model.py::test_autovc_bf16_b64_vs_oracle uses, with the same
metrics (outputs rel-Frobenius / rel-inf, losses, per-parameter gradient rel-Frobenius).  The GPU
bf16 bars of that test are set from this measurement, not from the GPU result.

  python tools/bf16_drift.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from autoformer_amd.detinit import det_inputs  # noqa: E402
from oracle import autovc_cpu as O  # noqa: E402


def rel_frob(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def rel_inf(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)


_LSTM = O.lstm


def _lstm_bf16_operands(x, sd, pre, hidden, layers, bidir, training=True):
    """torch.lstm under CPU autocast runs in bf16 end to end and its backward loses ~13x of the
    gradient magnitude upstream of the decoder's lstm2 (measured): the recurrences are emulated the
    way the GPU computes them instead -- bf16-rounded inputs and weights, fp32 gates, cell state and
    accumulation."""
    with torch.autocast("cpu", enabled=False):
        keys = [k for k in sd if k.startswith(pre + ".")]
        saved = {k: sd[k] for k in keys}
        try:
            for k in keys:
                if "weight" in k:
                    sd[k] = _RoundBF16.apply(saved[k])
            return _LSTM(_RoundBF16.apply(x.float()), sd, pre, hidden, layers, bidir, training)
        finally:
            sd.update(saved)


class _RoundBF16(torch.autograd.Function):
    """Round to bf16 in the forward, identity gradient (the operand cast of a bf16 GEMM)."""

    @staticmethod
    def forward(ctx, t):
        return t.bfloat16().float()

    @staticmethod
    def backward(ctx, g):
        return g


def run(bf16, golden=None):
    O.lstm = _lstm_bf16_operands if bf16 else _LSTM
    B, T, freq = 64, 128, 16
    if golden is not None:  # the B=2 golden inputs (tests/golden/autovc_T*.npz)
        freq = int(golden["freq"])
        xt, et = torch.from_numpy(golden["x"]), torch.from_numpy(golden["emb"])
    else:
        x, e = det_inputs(B, T, seed=21)
        xt, et = torch.from_numpy(x), torch.from_numpy(e)
    sd = O.make_state(O.autovc_spec())
    with torch.autocast("cpu", dtype=torch.bfloat16, enabled=bf16):
        losses, total, outs = O.step_losses(lambda a, b, c: O.autovc_forward(sd, a, b, c, freq=freq), xt, et)
    total.backward()
    grads = {k: v.grad.detach().clone() for k, v in sd.items() if v.requires_grad and v.grad is not None}
    return [o.detach().float() for o in outs], [float(l) for l in losses], grads


if __name__ == "__main__":
    torch.set_num_threads(min(8, torch.get_num_threads()))
    if len(sys.argv) > 1:  # B=2 goldens: the output drift only (tests/test_gpu_model.py::test_autovc_bf16_loose)
        for name in sys.argv[1:]:
            g = np.load(os.path.join(ROOT, "tests", "golden", name))
            o32, _, _ = run(False, g)
            o16, _, _ = run(True, g)
            print(f"{name} (B=2): oracle bf16 vs fp32 mel_psnt rel-Frobenius {rel_frob(o16[1], o32[1]):.3e} "
                  f"rel-inf {rel_inf(o16[1], o32[1]):.3e}, mel {rel_frob(o16[0], o32[0]):.3e} / "
                  f"{rel_inf(o16[0], o32[0]):.3e}")
        sys.exit(0)
    o32, l32, g32 = run(False)
    o16, l16, g16 = run(True)
    gmax = max(float(g.norm()) for g in g32.values())
    res = {"mel_psnt_frob": rel_frob(o16[1], o32[1]), "mel_psnt_inf": rel_inf(o16[1], o32[1]),
           "mel_frob": rel_frob(o16[0], o32[0]), "mel_inf": rel_inf(o16[0], o32[0]),
           "loss_rtol": max(abs(a - b) / abs(b) for a, b in zip(l16, l32))}
    rels, zeros = [], []
    for k, g in g32.items():
        if float(g.norm()) < 1e-6 * gmax:
            zeros.append((float(g16[k].norm()) / gmax, k))
        else:
            rels.append((rel_frob(g16[k], g), k))
    rels.sort(reverse=True)
    res["grad_frob"] = rels[0][0]
    res["zero_grad_abs"] = max(zeros)[0] if zeros else 0.0
    print("oracle bf16-autocast vs oracle fp32 (B=64 T=128 freq=16, det_inputs seed 21): "
          + " ".join(f"{k} {v:.3e}" for k, v in res.items()))
    print("worst gradients: " + ", ".join(f"{n} {r:.3e}" for r, n in rels[:8]))
    print(f"median gradient rel-Frobenius {rels[len(rels) // 2][0]:.3e} over {len(rels)} tensors; "
          f"{len(zeros)} analytically-zero")
    if os.environ.get("DEBUG"):
        for r, n in rels[:4] + rels[-4:]:
            print(n, float(g32[n].norm()), float(g16[n].norm()), r)
