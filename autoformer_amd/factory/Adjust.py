"""Adjust (/root/reference/factory/Adjust.py:7-43): refines a speaker embedding from the
utterance it belongs to — cat(mel, emb broadcast) -> 3 x ReLU(BN(conv5 -> 512)) ->
LSTM(512, 768, 3 layers) -> last step -> Linear(768 -> 256) -> L2 normalise.

HIP path: enc_conv0 (concat + conv + BN epilogue; the embedding gradient as a per-utterance
time sum when the embedding itself is trained), conv_bn x2, three LSTM layers, step
select, linear, row normalisation (variants.hip)."""
import torch.nn as nn

from .. import kernels as K
from .. import layers as Lyr
from .. import variants as V
from .AutoVC import _conv_bn_block, _frames
from .Norm import LinearNorm, LSTMParams


class Adjust(nn.Module):
    def __init__(self, dim_emb, dim_cell=768):
        super().__init__()
        self.convolutions = nn.ModuleList(
            [_conv_bn_block(80 + dim_emb if i == 0 else 512, 512, "relu") for i in range(3)])
        self.lstm = LSTMParams(512, hidden_size=dim_cell, num_layers=3, batch_first=True)
        self.embedding = LinearNorm(dim_cell, 256)
        self._convs = [Lyr.ConvBNCore(s[0].conv, s[1], K.ACT_RELU) for s in self.convolutions]
        self._lstm = [Lyr.LSTMLayerCore(self.lstm, layer) for layer in range(3)]
        self._lin = Lyr.PackCache()

    def forward(self, x, emb, stat_updates=1):
        """stat_updates = 2: this call stands for two reference calls on identical inputs (the
        outputs are identical; each BatchNorm's running statistics move twice, as there)."""
        K.require_device(x, emb)
        mel, B, T = _frames(x)
        for core in self._convs:
            core.stat_updates = stat_updates
        try:
            h = Lyr.enc_conv0(self._convs[0], mel, emb.contiguous(), B, T)
            for core in self._convs[1:]:
                h = Lyr.conv_bn(core, h, B, T)
        finally:
            for core in self._convs:
                core.stat_updates = 1
        h = Lyr.lstm(self.lstm, self._lstm, h, B, T)
        last = V.step_select(h, B, T, T - 1)
        lin = self.embedding.linear_layer
        return V.rownorm(Lyr.linear(last, lin.weight, lin.bias, self._lin))
