"""Autograd ops of the AdaIN ("2") and speaker-embedding-adjust ("_Adjust") variants
(SURVEY.md §8(f) rank 4), each a HIP kernel pair from variants.hip:

  moments(x)           -> (2,) [x.mean(), x.std()]    factory/AutoVC2.py:58-60 (features)
  adain(x, mu, sigma)                                  factory/Norm.py:84-91
  step_select(h, ...)  nn.LSTM output [:, t, :]        factory/Adjust.py:39
  rownorm(e)           e / ||e||_2 per row             factory/Adjust.py:40-42

Tensors may have any shape (moments / AdaIN are whole-tensor ops, so the frame-major
layout the build keeps gives the reference's (B, C, T) results).
"""
import torch

from . import kernels as K


class _MomentsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        mom = K.moments(x)
        ctx.save_for_backward(x, mom)
        return mom

    @staticmethod
    def backward(ctx, dmom):
        x, mom = ctx.saved_tensors
        dmom = dmom.contiguous()
        return K.moments_bwd(x, mom, dmom[0], dmom[1])


def moments(x):
    """Differentiable (2,) tensor [mean, std]; the reference's features are [m[0], m[1]]."""
    return _MomentsFn.apply(x)


class _AdaINFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mu, sigma):
        x = x.contiguous()
        mom = K.moments(x)
        ctx.save_for_backward(x, mom, sigma)
        return K.adain_fwd(x, mom, mu, sigma)

    @staticmethod
    def backward(ctx, g):
        x, mom, sigma = ctx.saved_tensors
        dx, dmu, dsig = K.adain_bwd(g.contiguous(), x, mom, sigma)
        return (dx if ctx.needs_input_grad[0] else None, dmu if ctx.needs_input_grad[1] else None,
                dsig if ctx.needs_input_grad[2] else None)


def _scalar(v, like):
    if isinstance(v, torch.Tensor):
        if v.numel() != 1:
            raise ValueError(f"AdaIN statistics must be scalars, got shape {tuple(v.shape)}")
        return v.reshape(()).to(like.device, torch.float32)
    return torch.tensor(float(v), device=like.device)


def adain(content, mu, std):
    """AdaIN.forward (Norm.py:84-91): (c - c.mean()) / c.std() * std + mu."""
    return _AdaINFn.apply(content, _scalar(mu, content), _scalar(std, content))


class _StepSelectFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, B, T, t):
        ctx.dims = (B, T, t)
        return K.step_select(h.contiguous(), B, T, t)

    @staticmethod
    def backward(ctx, d):
        B, T, t = ctx.dims
        return K.step_scatter(d.contiguous(), B, T, t), None, None, None


def step_select(h, B, T, t):
    """Frame-major (B*T, C) -> (B, C) at time step t."""
    return _StepSelectFn.apply(h, B, T, t)


class _RowNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y, norms = K.rownorm_fwd(x.contiguous())
        ctx.save_for_backward(y, norms)
        return y

    @staticmethod
    def backward(ctx, dy):
        y, norms = ctx.saved_tensors
        return K.rownorm_bwd(dy.contiguous(), y, norms)


def rownorm(x):
    """x.div(x.norm(p=2, dim=-1, keepdim=True)) for a 2-D x (Adjust.py:40-42)."""
    return _RowNormFn.apply(x)
