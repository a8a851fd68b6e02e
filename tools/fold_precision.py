"""fp32 fold vs unfold error against a float64 torch reference of the decoder lstm1 (concat input)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import autoformer_amd as A  # noqa: E402
from autoformer_amd import layers as Lyr  # noqa: E402
from autoformer_amd.factory.Norm import LSTMParams  # noqa: E402

DEV = "cuda:0"
A.set_compute("fp32")
torch.manual_seed(0)
B, T, nc, cd, de, H = 2, 128, 8, 88, 256, 512
mod = LSTMParams(cd + de, H, 1, batch_first=True).to(DEV)
core = Lyr.LSTMLayerCore(mod, 0)
codes0 = torch.randn(B, nc * cd, device=DEV)
emb0 = torch.randn(B, de, device=DEV)
dh = torch.randn(B * T, H, device=DEV)
# float64 reference
ref = torch.nn.LSTM(cd + de, H, 1, batch_first=True).double()
with torch.no_grad():
    for n, p in ref.named_parameters():
        p.copy_(getattr(mod, n).detach().cpu().double())
c64 = codes0.cpu().double().requires_grad_(True)
e64 = emb0.cpu().double().requires_grad_(True)
x64 = torch.cat([c64.view(B, nc, 1, cd).expand(B, nc, T // nc, cd).reshape(B, T, cd),
                 e64.view(B, 1, de).expand(B, T, de)], -1)
h64, _ = ref(x64)
h64.backward(dh.cpu().double().view(B, T, H))
for fold in (False, True):
    codes = codes0.clone().requires_grad_(True)
    emb = emb0.clone().requires_grad_(True)
    for p in mod.parameters():
        p.grad = None
    if fold:
        h = Lyr.lstm1_folded(mod, core, codes, emb, B, T, nc, cd)
    else:
        h = Lyr.lstm(mod, [core], Lyr.dec_concat(codes, emb, B, T, nc, cd), B, T)
    h.backward(dh)
    torch.cuda.synchronize()
    Lyr.join_side()

    def rel(a, b):
        a, b = a.detach().cpu().double().reshape(-1), b.detach().reshape(-1)
        return float((a - b).norm() / b.norm()), float((a - b).abs().max() / b.abs().max())
    print("fold" if fold else "unfold", "h", rel(h, h64.reshape(B * T, H)), "dcodes", rel(codes.grad, c64.grad),
          "demb", rel(emb.grad, e64.grad), "dWih", rel(mod.weight_ih_l0.grad, ref.weight_ih_l0.grad),
          "dWhh", rel(mod.weight_hh_l0.grad, ref.weight_hh_l0.grad), flush=True)
