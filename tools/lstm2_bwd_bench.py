"""Isolated timing of the decoder lstm2 backward (B=64, T=128, H=1024, bf16): the two-layer wavefront
launch (avc_lstm2_bwd) vs two single-layer persistent launches + the dX1 GEMM, plus the wavefront's
per-tick stamps (avc_lstm_trace: step start, exchange + products done, published).

  python tools/lstm2_bwd_bench.py [reps]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import autoformer_amd as A  # noqa: E402
from autoformer_amd import _lib  # noqa: E402
from autoformer_amd import kernels as K  # noqa: E402
from autoformer_amd import layers as Ly  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    A.set_compute("bf16")
    B, T, H = 64, 128, 1024
    dev = "cuda:0"
    torch.manual_seed(0)
    mod = torch.nn.LSTM(512, H, 2, batch_first=True).to(dev)
    cores = [Ly.LSTMLayerCore(mod, layer) for layer in range(2)]
    x = (torch.randn(B * T, 512, device=dev) * 0.5).requires_grad_(True)
    Ly.set_grad_sink(False)
    y = Ly.lstm(mod, cores, x, B, T)
    gy = torch.randn(B * T, H, device=dev) * 0.1
    fn = y.grad_fn
    saved = fn.saved  # ((c0, g0), (c1, g1))
    (cs0, gs0), (cs1, gs1) = saved
    wt0 = cores[0].packs()[3]
    _, _, _, wt1, wti1 = cores[1].packs()
    h0 = fn.saved_tensors[1]
    h1 = fn.saved_tensors[2]

    def wave():
        return K.lstm2_bwd(gy, cs0, gs0, cs1, gs1, wt0, wti1, wt1, B, T, H)

    def wave16():  # the step's form (ABI 28): bf16 dG + per-group bias partials
        return K.lstm2_bwd(gy, cs0, gs0, cs1, gs1, wt0, wti1, wt1, B, T, H, fp32=False, db=True)

    def two():
        dg1 = K.lstm_bwd(gy, h1, cs1, gs1, None, wt1, B, T, H, 1)
        dh0 = torch.empty(B * T, H, device=dev)
        K.gemm(B * T, H, 4 * H, Ly.operand(dg1, 4 * H), Ly.operand(wti1, 4 * H), dh0)
        return K.lstm_bwd(dh0, h0, cs0, gs0, None, wt0, B, T, H, 1), dg1

    def ev(f):
        f()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            f()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        return min(ts), sorted(ts)[len(ts) // 2]

    for name, f in (("wavefront", wave), ("wavefront bf16 + db", wave16), ("two launches + GEMM", two),
                    ("wavefront", wave), ("wavefront bf16 + db", wave16), ("two launches + GEMM", two)):
        mn, md = ev(f)
        print(f"{name:22s} min {mn:7.1f} us  med {md:7.1f} us", flush=True)
    (a0, a1), (b0, b1) = wave(), two()
    torch.cuda.synchronize()
    rel = lambda p, q: ((p.double() - q.double()).norm() / q.double().norm()).item()  # noqa: E731
    print(f"dG0 rel {rel(a0, b0):.2e}  dG1 rel {rel(a1, b1):.2e}")
    # per-tick stamps of the wavefront
    ng = (B + 15) // 16
    nwg = ng * (H // 16)
    tr = torch.zeros(nwg * T * 4, dtype=torch.int64, device=dev)
    _lib.call("avc_lstm_trace", tr.data_ptr())
    wave()
    torch.cuda.synchronize()
    _lib.call("avc_lstm_trace", None)
    st = tr.view(nwg, T, 4).cpu().numpy().astype(np.float64) / 100.0  # 100 MHz -> us
    ks = slice(1, T - 1)
    wait_prod = (st[:, ks, 2] - st[:, ks, 0]).mean()
    tail = (st[:, ks, 3] - st[:, ks, 2]).mean()
    period = np.diff(st[:, :, 0], axis=1)[:, 1:-1].mean()
    print(f"wavefront per tick: start -> products reduced {wait_prod:.2f} us, -> published {tail:.2f} us, "
          f"period {period:.2f} us")
    # stamp 1 = the group's flags all seen (after the poll's barrier): the tick's wait vs its gather
    wait = (st[:, ks, 1] - st[:, ks, 0]).mean()
    gath = (st[:, ks, 2] - st[:, ks, 1]).mean()
    print(f"  start -> flags seen {wait:.2f} us, flags seen -> products reduced {gath:.2f} us")
    # producer skew: per group and tick, the members' publish stamps (flag raised just before stamp 3)
    grp = np.arange(nwg) % ng
    skew, hop = [], []
    for g in range(ng):
        m = grp == g
        for k in range(1, T - 2):
            pub = st[m, k, 3]
            seen = st[m, k + 1, 1]
            skew.append(pub.max() - np.median(pub))
            hop.append(seen.min() - pub.max())
    skew, hop = np.array(skew), np.array(hop)
    print(f"  producer skew (last publish - median publish) mean {skew.mean():.2f} us, p90 {np.percentile(skew, 90):.2f}; "
          f"last publish -> first consumer's flags seen {hop.mean():.2f} us")


if __name__ == "__main__":
    main()
