"""Drop-in DeepConvDiscNet backed by the pcadv linear kernels
(models/discriminator.py:30-51): five 1x1 Conv1d layers on B x C x 1 with
LeakyReLU(0.2), then Linear(64, output_dim).  Same state_dict as the reference."""
from __future__ import annotations

import torch.nn as nn

from .ops import ACT_LRELU, ACT_NONE, LinearFunction

__all__ = ["DeepConvDiscNet"]


class DeepConvDiscNet(nn.Module):
    def __init__(self, input_dim, output_dim):
        super().__init__()
        self.conv1 = nn.Conv1d(input_dim, 512, 1)
        self.conv2 = nn.Conv1d(512, 256, 1)
        self.conv3 = nn.Conv1d(256, 256, 1)
        self.conv4 = nn.Conv1d(256, 64, 1)
        self.conv5 = nn.Conv1d(64, 64, 1)
        self.fc = nn.Linear(64, output_dim)
        self.leaky_relu = nn.LeakyReLU(negative_slope=0.2, inplace=True)

    def forward(self, x):
        h = x.contiguous()
        for conv in (self.conv1, self.conv2, self.conv3, self.conv4, self.conv5):
            h = LinearFunction.apply(h, conv.weight, conv.bias, ACT_LRELU, None, 0.0)
        return LinearFunction.apply(h, self.fc.weight, self.fc.bias, ACT_NONE, None, 0.0)
