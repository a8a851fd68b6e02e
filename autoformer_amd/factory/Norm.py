"""Parameter containers with the reference's names, shapes and initialisation.

Mirrors /root/reference/factory/Norm.py (ConvNorm :4-37, LinearNorm :40-50, GroupNorm
:53-60, PatchEmbed :63-82) so that ``state_dict`` keys match exactly.  These modules
hold parameters only; the computation is done by autoformer_amd.layers on HIP kernels,
driven by the parent model's forward.
"""
import torch.nn as nn


class ConvNorm(nn.Module):
    def __init__(self, in_channels, out_channels, kernel_size=5, stride=1, padding=None, dilation=1, bias=True,
                 w_init_gain="linear"):
        super().__init__()
        if padding is None:
            assert kernel_size % 2 == 1
            padding = int(dilation * (kernel_size - 1) / 2)
        if stride != 1 or dilation != 1:
            raise NotImplementedError("only stride=1, dilation=1 convolutions are on the AutoVC path")
        self.conv = nn.Conv1d(in_channels, out_channels, kernel_size=kernel_size, stride=stride, padding=padding,
                              dilation=dilation, bias=bias)
        nn.init.xavier_uniform_(self.conv.weight, gain=nn.init.calculate_gain(w_init_gain))

    def forward(self, signal):  # pragma: no cover - the parent model drives the kernels
        raise RuntimeError("ConvNorm is driven by its parent model's HIP forward")


class LinearNorm(nn.Module):
    def __init__(self, in_dim, out_dim, bias=True, w_init_gain="linear"):
        super().__init__()
        self.linear_layer = nn.Linear(in_dim, out_dim, bias=bias)
        nn.init.xavier_uniform_(self.linear_layer.weight, gain=nn.init.calculate_gain(w_init_gain))

    def forward(self, x):  # pragma: no cover
        raise RuntimeError("LinearNorm is driven by its parent model's HIP forward")


class GroupNorm(nn.GroupNorm):
    """Group Normalization with 1 group (Norm.py:53-60)."""

    def __init__(self, num_channels, **kwargs):
        super().__init__(1, num_channels, **kwargs)


class PatchEmbed(nn.Module):
    """Conv1d patch embedding (Norm.py:63-82)."""

    def __init__(self, patch_size=5, stride=1, padding=2, in_chans=336, embed_dim=512):
        super().__init__()
        self.proj = nn.Conv1d(in_chans, embed_dim, kernel_size=patch_size, stride=stride, padding=padding)
        self.norm = nn.Identity()


class LSTMParams(nn.Module):
    """Parameters of nn.LSTM(batch_first=True) under the same names (weight_ih_l0, ...,
    *_reverse) and with nn.LSTM's U(-1/sqrt(H), 1/sqrt(H)) initialisation.  The recurrence
    runs in lstm.hip; ``flatten_parameters`` (a cuDNN weight-packing hint in the reference,
    AutoVC.py:54) is a no-op here."""

    def __init__(self, input_size, hidden_size, num_layers=1, batch_first=True, bidirectional=False):
        super().__init__()
        import math

        import torch

        assert batch_first
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        self.bidirectional = bidirectional
        self.batch_first = True
        dirs = 2 if bidirectional else 1
        k = 1.0 / math.sqrt(hidden_size)
        for layer in range(num_layers):
            lin = input_size if layer == 0 else hidden_size * dirs
            for sfx in (["", "_reverse"] if bidirectional else [""]):
                for name, shape in (("weight_ih", (4 * hidden_size, lin)), ("weight_hh", (4 * hidden_size, hidden_size)),
                                    ("bias_ih", (4 * hidden_size,)), ("bias_hh", (4 * hidden_size,))):
                    p = nn.Parameter(torch.empty(*shape))
                    nn.init.uniform_(p, -k, k)
                    self.register_parameter(f"{name}_l{layer}{sfx}", p)

    def flatten_parameters(self):
        return None

    def forward(self, *a, **k):  # pragma: no cover
        raise RuntimeError("LSTMParams is driven by its parent model's HIP forward")


class AdaIN(nn.Module):
    """AdaIN (Norm.py:84-91): (content - content.mean()) / content.std() * std + mu, with
    whole-tensor statistics; HIP moments + apply kernels (variants.hip)."""

    def forward(self, content, mu, std):
        from .. import variants as V

        return V.adain(content, mu, std)


class IN(nn.Module):
    """IN (Norm.py:94-104): ((content - mu) / std, mu expanded, std)."""

    def forward(self, content):
        import torch

        from .. import variants as V

        m = V.moments(content)
        y = V.adain(content, torch.zeros((), device=content.device), torch.ones((), device=content.device))
        return y, m[0].expand(content.size()), m[1]
