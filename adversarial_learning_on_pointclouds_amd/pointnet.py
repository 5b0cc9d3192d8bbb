"""Drop-in PointNet modules backed by the pcadv HIP kernels.

Same class names, constructor arguments, forward signatures, return tuples and
state_dict keys/shapes as the reference's models/pointnet.py, so checkpoints
load in either direction and utils/trainer.py-style loops run unchanged.
The compute runs in libpcadv.so; there is no eager-PyTorch fallback.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .ops import (ACT_NONE, ACT_RELU, ConvMaxFunction, LinearFunction, PointFeatFunction,
                  PointwiseFunction, RegularizerFunction, TransformFunction)

__all__ = ["PointNetfeat", "PointNetCls", "STN3d", "STNkd", "feature_transform_regularizer"]


class STNkd(nn.Module):
    """k x k transform regressor (models/pointnet.py:46-79): relu(conv1..conv3),
    ReLU then max over points, relu(fc1), relu(fc2), fc3 + identity."""

    def __init__(self, k=64):
        super().__init__()
        self.conv1 = nn.Conv1d(k, 64, 1)
        self.conv2 = nn.Conv1d(64, 128, 1)
        self.conv3 = nn.Conv1d(128, 1024, 1)
        self.fc1 = nn.Linear(1024, 512)
        self.fc2 = nn.Linear(512, 256)
        self.fc3 = nn.Linear(256, k * k)
        self.relu = nn.ReLU()
        self.k = k

    def forward_points(self, xp):
        """xp: B x N x k point-major -> B x k x k."""
        h = PointwiseFunction.apply(xp, self.conv1.weight, self.conv1.bias, ACT_RELU)
        h = PointwiseFunction.apply(h, self.conv2.weight, self.conv2.bias, ACT_RELU)
        g = ConvMaxFunction.apply(h, self.conv3.weight, self.conv3.bias, True)
        f = LinearFunction.apply(g, self.fc1.weight, self.fc1.bias, ACT_RELU, None, 0.0)
        f = LinearFunction.apply(f, self.fc2.weight, self.fc2.bias, ACT_RELU, None, 0.0)
        t = LinearFunction.apply(f, self.fc3.weight, self.fc3.bias, ACT_NONE, None, 0.0, self.k)
        return t.view(-1, self.k, self.k)

    def forward(self, x):
        """x: B x k x N (the reference layout)."""
        return self.forward_points(x.transpose(1, 2).contiguous())


class STN3d(STNkd):
    """3 x 3 input transform (models/pointnet.py:14-43)."""

    def __init__(self):
        super().__init__(k=3)


class PointNetfeat(nn.Module):
    """models/pointnet.py:81-137.  forward(x: B x 3 x N) -> (global B x 1024, trans_feat)."""

    def __init__(self, global_feat=True, feature_transform=False):
        super().__init__()
        self.conv1 = nn.Conv1d(3, 64, 1)
        self.conv2 = nn.Conv1d(64, 64, 1)
        self.conv3 = nn.Conv1d(64, 128, 1)
        self.conv4 = nn.Conv1d(128, 1024, 1)
        self.global_feat = global_feat
        self.feature_transform = feature_transform
        if self.feature_transform:
            self.fstn = STNkd(k=64)

    def forward_points(self, pts, with_pointfeat=False):
        """pts: C x N x 3 (point-major, as PointNetCls receives it) ->
        (global C x 1024, trans_feat or None), plus the point features (C x N x 64,
        conv2's output after the optional feature transform) with_pointfeat."""
        if self.feature_transform or with_pointfeat:
            # models/pointnet.py:115-130 layer by layer (point-wise kernels, the
            # STNkd(64) feature transform if on, the sparse max-pool backward)
            x = PointwiseFunction.apply(pts.contiguous(), self.conv1.weight, self.conv1.bias,
                                        ACT_RELU)
            x = PointwiseFunction.apply(x, self.conv2.weight, self.conv2.bias, ACT_RELU)
            trans_feat = None
            if self.feature_transform:
                trans_feat = self.fstn.forward_points(x)
                x = TransformFunction.apply(x, trans_feat)
            pointfeat = x
            x = PointwiseFunction.apply(x, self.conv3.weight, self.conv3.bias, ACT_RELU)
            g = ConvMaxFunction.apply(x, self.conv4.weight, self.conv4.bias, False)
            return (g, trans_feat, pointfeat) if with_pointfeat else (g, trans_feat)
        gmax, gidx = PointFeatFunction.apply(
            pts.contiguous(), self.conv1.weight, self.conv1.bias, self.conv2.weight,
            self.conv2.bias, self.conv3.weight, self.conv3.bias, self.conv4.weight,
            self.conv4.bias)
        self.last_argmax = gidx
        return gmax, None

    def forward(self, x):
        # the reference receives B x C x N; the kernels read the point-major
        # B x N x 3 layout, which is a free view when x came from a transpose.
        if self.global_feat:
            return self.forward_points(x.transpose(1, 2))
        # models/pointnet.py:133-137: the global feature repeated over the points,
        # then the point features: B x (1024 + 64) x N
        n_pts = x.size(2)
        g, trans_feat, pointfeat = self.forward_points(x.transpose(1, 2), with_pointfeat=True)
        return torch.cat([g.unsqueeze(2).expand(-1, -1, n_pts), pointfeat.transpose(1, 2)],
                         1), trans_feat


class PointNetCls(nn.Module):
    """models/pointnet.py:186-203.  forward(x: B x N x 3) ->
    (logits B x k, x_global B x 1024 x 1, trans_feat)."""

    def __init__(self, k=3, feature_transform=False):
        super().__init__()
        self.feature_transform = feature_transform
        self.feat = PointNetfeat(global_feat=True, feature_transform=feature_transform)
        self.fc1 = nn.Linear(1024, 512)
        self.fc2 = nn.Linear(512, 256)
        self.fc3 = nn.Linear(256, k)
        self.dropout = nn.Dropout(p=0.3)
        self.relu = nn.ReLU()
        # optional queue of explicit dropout masks (B x 256 {0,1}) for parity runs
        self.dropout_masks = []

    def _dropout_mask(self, B, device):
        if not self.training or self.dropout.p == 0.0:
            return None
        if self.dropout_masks:
            return self.dropout_masks.pop(0).to(device=device, dtype=torch.float32).contiguous()
        return (torch.rand(B, 256, device=device) >= self.dropout.p).float()

    def forward(self, x):
        x_global, trans_feat = self.feat.forward_points(x)
        h = LinearFunction.apply(x_global, self.fc1.weight, self.fc1.bias, ACT_RELU, None, 0.0)
        mask = self._dropout_mask(x.shape[0], x.device)
        h = LinearFunction.apply(h, self.fc2.weight, self.fc2.bias, ACT_RELU, mask,
                                 float(self.dropout.p))
        out = LinearFunction.apply(h, self.fc3.weight, self.fc3.bias, ACT_NONE, None, 0.0)
        return out, x_global.unsqueeze(2), trans_feat


def feature_transform_regularizer(trans):
    """mean_b ||T T^T - I||_F (models/pointnet.py:345-353) on the HIP device."""
    return RegularizerFunction.apply(trans)
