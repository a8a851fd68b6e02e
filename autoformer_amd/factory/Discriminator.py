"""Discriminator of train_with_discriminator.py — drop-in for
/root/reference/factory/Discriminator.py (same constructor, forward(x (B, crop_len, 80))
-> (B, 1) probabilities, same state_dict).

The reference runs Conv1d with TIME as channels (176 -> 88 -> 44 -> 22) over the 80
mel bins, LeakyReLU(0.01) BEFORE each BatchNorm, flatten (channel-major, 1628), Linear,
Sigmoid (Discriminator.py:18-29).  Here the input is transposed once to bin-major frames
(B*80, 176) so every conv is the same windowed GEMM as AutoVC's (taps 3, no padding); the
flatten order difference is absorbed by permuting dense1's weight (and its gradient).
The whole network is one autograd function of HIP kernels.
"""
import torch
import torch.nn as nn

from .. import kernels as K
from .. import layers as Lyr


def _transpose_b(x, B, R, C):
    return Lyr._transpose_batched(x, B, R, C)


class _DiscFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mod, *params):
        B, C0, L0 = x.shape
        c1, c2, c3, bn1, bn2, dense = mod.conv1, mod.conv2, mod.conv3, mod.bn1, mod.bn2, mod.dense1
        xt = _transpose_b(x.contiguous(), B, C0, L0).view(B * L0, C0)  # (B*80, 176) bins as frames
        # bf16 compute: the conv GEMMs read bf16 twins of their fp32 operands (one conversion pass
        # each; without them the fp32-operand GEMM paths ran: 0.55 ms per C5 step, measured)
        xt = K.twin(xt)
        Wf1, _ = Lyr.conv_packs(mod._c[0], c1.weight)
        Wf2, _ = Lyr.conv_packs(mod._c[1], c2.weight)
        Wf3, _ = Lyr.conv_packs(mod._c[2], c3.weight)
        y1, L1 = Lyr.conv_fwd(xt, B, L0, c1.weight, c1.bias, 0, Wf1)
        a1 = K.twin(K.act_fwd(y1, K.ACT_LEAKY))
        y2, L2 = Lyr.conv_fwd(a1, B, L1, c2.weight, c2.bias, 0, Wf2)
        z2 = K.act_fwd(y2, K.ACT_LEAKY)
        st1 = mod._bn(bn1, z2)
        a2 = K.bn_apply(z2, st1[2], st1[3], K.ACT_NONE)
        y3, L3 = Lyr.conv_fwd(a2, B, L2, c3.weight, c3.bias, 0, Wf3)
        z3 = K.act_fwd(y3, K.ACT_LEAKY)
        st2 = mod._bn(bn2, z3)
        a3 = K.bn_apply(z3, st2[2], st2[3], K.ACT_NONE)
        C3 = c3.weight.shape[0]
        # dense1 + sigmoid: dense1.weight is (1, C3*L3) channel-major, a3's rows are (l, c)
        # bin-major; the kernel indexes the weight through that permutation (disc.hip)
        wd = dense.weight.detach()
        p = K.disc_dense_fwd(a3, wd, dense.bias, B, L3, C3)
        ctx.mod = mod
        ctx.dims = (B, C0, L0, L1, L2, L3, C3)
        ctx.stats = (st1, st2)
        ctx.save_for_backward(xt, a1, z2, a2, z3, a3, wd, p)
        ctx.twins = tuple(getattr(t, "_bf16", None) for t in (xt, a1, a2))
        return p

    @staticmethod
    def backward(ctx, dp):
        xt, a1, z2, a2, z3, a3, wd, p = ctx.saved_tensors
        for t, tw in zip((xt, a1, a2), ctx.twins):
            K.attach_twin(t, tw)
        mod = ctx.mod
        B, C0, L0, L1, L2, L3, C3 = ctx.dims
        (m1, r1, _, _), (m2, r2, _, _) = ctx.stats
        c1, c2, c3, bn1, bn2, dense = mod.conv1, mod.conv2, mod.conv3, mod.bn1, mod.bn2, mod.dense1
        da3, d_dense_w, d_dense_b = K.disc_dense_bwd(dp.contiguous(), p, a3, wd, B, L3, C3)
        dz3, dg2, db2, _ = K.bn_bwd(da3.view(B * L3, C3), a3, z3, m2, r2, bn2.weight, K.ACT_NONE, need_dbias=False)
        dy3 = K.act_bwd(dz3, z3, K.ACT_LEAKY)
        _, Wd2 = Lyr.conv_packs(mod._c[1], c2.weight)
        _, Wd1 = Lyr.conv_packs(mod._c[0], c1.weight)
        # conv3's 22 output channels: dy3 and the data-gradient pack zero-padded to a multiple of 4,
        # so both conv3 gradient products take the vectorised GEMM kernels (22-wide rows ran on the
        # generic kernel: 2 x 85 us per C5 step)
        C2, C3p = c3.weight.shape[1], -(-C3 // 4) * 4
        w3 = c3.weight
        dy3p = K.pad_cols(dy3, C3p, K.compute())
        Wd3 = mod._c3d.get([w3], lambda: K.conv_pack_slice(w3.detach(), 0, C2, C3p, 3, K.compute()))
        dWf3 = torch.empty(C3p, 3 * C2, device=p.device)
        K.gemm(C3p, 3 * C2, B * L3, Lyr.operand(dy3p, C3p, kstrided=True),
               Lyr.operand(a2, C2, kstrided=True, window=(3, 0, L3, L2, C2)), dWf3,
               split_k=K.auto_split_k(C3p, 3 * C2, B * L3))
        dW3 = K.conv_grad_unpack(dWf3[:C3], C3, C2, 3)
        db3 = K.colsum(dy3, B * L3, C3)
        da2 = torch.empty(B * L2, C2, device=p.device)
        K.gemm(B * L2, C2, 3 * C3p, Lyr.operand(dy3p, C3p, window=(3, 2, L2, L3, C3p)), Lyr.operand(Wd3, 3 * C3p), da2)
        dz2, dg1, db1, _ = K.bn_bwd(da2, a2, z2, m1, r1, bn1.weight, K.ACT_NONE, need_dbias=False)
        dy2 = K.twin(K.act_bwd(dz2, z2, K.ACT_LEAKY))
        dW2 = Lyr.conv_wgrad(dy2, a1, B, L1, L2, c2.weight, 0)
        dbc2 = K.colsum(dy2, B * L2, c2.weight.shape[0])
        da1 = Lyr.conv_dgrad(dy2, B, L1, L2, c2.weight, 0, Wd2)
        dy1 = K.twin(K.act_bwd(da1, a1, K.ACT_LEAKY))
        dW1 = Lyr.conv_wgrad(dy1, xt, B, L0, L1, c1.weight, 0)
        dbc1 = K.colsum(dy1, B * L1, c1.weight.shape[0])
        dx = None
        if ctx.needs_input_grad[0]:
            dxt = Lyr.conv_dgrad(dy1, B, L0, L1, c1.weight, 0, Wd1)
            dx = _transpose_b(dxt, B, L0, C0).view(B, C0, L0)
        return (dx, None, dW1, dbc1, dW2, dbc2, dW3, db3, dg1, db1, dg2, db2, d_dense_w, d_dense_b)


class Discriminator(nn.Module):
    def __init__(self, crop_len=176, dim_neck=44):
        super().__init__()
        self.conv1 = nn.Conv1d(crop_len, 2 * dim_neck, 3)
        self.conv2 = nn.Conv1d(2 * dim_neck, dim_neck, 3)
        self.conv3 = nn.Conv1d(dim_neck, int(dim_neck / 2), 3)
        self.leaky_relu = nn.LeakyReLU()
        self.bn1 = nn.BatchNorm1d(dim_neck)
        self.bn2 = nn.BatchNorm1d(int(dim_neck / 2))
        self.flatten = nn.Flatten()
        self.dense1 = nn.Linear(1628, 1)
        self.sigmoid = nn.Sigmoid()
        self._c = [Lyr.PackCache() for _ in range(3)]
        self._c3d = Lyr.PackCache()  # conv3 data-gradient pack, output channels padded

    def _bn(self, bn, z):
        M, C = z.shape
        if bn.training:
            part = K.bn_stats(z, M, C)
            nbt = bn.num_batches_tracked if bn.track_running_stats else None
            return K.bn_finalize(part, M, C, bn.weight, bn.bias, bn.running_mean, bn.running_var, nbt,
                                 bn.momentum if bn.momentum is not None else 0.1, bn.eps)
        return K.bn_eval(bn.running_mean, bn.running_var, bn.weight, bn.bias, bn.eps)

    def forward(self, x):
        K.require_device(x)
        ps = [self.conv1.weight, self.conv1.bias, self.conv2.weight, self.conv2.bias, self.conv3.weight,
              self.conv3.bias, self.bn1.weight, self.bn1.bias, self.bn2.weight, self.bn2.bias, self.dense1.weight,
              self.dense1.bias]
        return _DiscFn.apply(x, self, *ps)
