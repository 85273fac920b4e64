"""ResNet family with the reference's exact topology, parameter names and initialisation.

* ``ResNet34``  — R/ResNet/pytorch/models/resnet34.py. NOTE: the reference's "ResNet-34" uses
  ``[2, 2, 2, 2]`` BasicBlocks (:38-41), i.e. ResNet-18 depth (11,689,512 params + fc), and a
  1x1 projection on the first block of *every* stage including conv2x (:69-75). Replicated
  as-is for checkpoint compatibility.
* ``ResNet50`` / ``ResNet152`` — R/ResNet/pytorch/models/resnet50.py / resnet152.py: V1
  bottleneck with the stride on the FIRST 1x1 (:101-107), projection on block 0 of each stage.

On GPU every conv -> BN -> (add) -> ReLU chain runs as one fused native op sequence
(conv epilogue BN statistics, single BN-apply pass with residual + ReLU).
"""
from __future__ import annotations

import torch.nn as tnn

from .. import nn
from .. import ops as F
from ..ops.conv import GradJoin


def _init(model):
    # R/ResNet/pytorch/models/resnet50.py:84-93
    for m in model.modules():
        if isinstance(m, tnn.Conv2d):
            tnn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
        elif isinstance(m, tnn.BatchNorm2d):
            tnn.init.constant_(m.weight, 1)
            tnn.init.constant_(m.bias, 0)


class BasicBlock(tnn.Module):
    def __init__(self, in_channels, out_channels, stride=1, downsample=False):
        super().__init__()
        self.conv1 = nn.Conv2d(in_channels, out_channels, 3, stride=stride, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(out_channels)
        self.conv2 = nn.Conv2d(out_channels, out_channels, 3, stride=1, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(out_channels)
        self.relu = nn.ReLU(inplace=True)
        self.projection = None
        self.downsample = downsample
        if downsample:
            self.projection = nn.Sequential(
                nn.Conv2d(in_channels, out_channels, 1, stride=stride, bias=False), nn.BatchNorm2d(out_channels))

    def forward(self, x):
        # GradJoin: the gradient of x from the shortcut (identity or projection) is folded into
        # conv1's dgrad epilogue instead of a separate autograd add (ops.conv.GradJoin)
        j = GradJoin() if F.native(x) else None
        out = F.conv_bn_act(x, self.conv1, self.bn1, "relu", join=j, join_role="consumer")
        rbn = None
        if self.downsample:  # projection BN folded into the block's last BN+add+ReLU pass
            identity, rbn = F.conv_bn_deferred(x, self.projection[0], self.projection[1], join=j, join_role="producer")
            rj = None
        else:
            identity, rj = x, j
        return F.conv_bn_act(out, self.conv2, self.bn2, "relu", residual=identity, residual_join=rj, residual_bn=rbn)


class BottleneckBlock(tnn.Module):
    def __init__(self, in_channels, out1, out2, stride=1, downsample=False):
        super().__init__()
        self.conv1 = nn.Conv2d(in_channels, out1, 1, stride=stride, bias=False)
        self.bn1 = nn.BatchNorm2d(out1)
        self.conv2 = nn.Conv2d(out1, out1, 3, stride=1, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(out1)
        self.conv3 = nn.Conv2d(out1, out2, 1, stride=1, bias=False)
        self.bn3 = nn.BatchNorm2d(out2)
        self.relu = nn.ReLU(inplace=True)
        self.projection = None
        self.downsample = downsample
        if downsample:
            self.projection = nn.Sequential(
                nn.Conv2d(in_channels, out2, 1, stride=stride, bias=False), nn.BatchNorm2d(out2))

    def forward(self, x):
        j = GradJoin() if F.native(x) else None
        out = F.conv_bn_act(x, self.conv1, self.bn1, "relu", join=j, join_role="consumer")
        out = F.conv_bn_act(out, self.conv2, self.bn2, "relu")
        # projection created after the main path: its backward runs first and stashes its dx;
        # its BatchNorm is applied inside bn3's BN+add+ReLU pass (ops.bn.conv_bn_deferred)
        rbn = None
        if self.downsample:
            identity, rbn = F.conv_bn_deferred(x, self.projection[0], self.projection[1], join=j, join_role="producer")
            rj = None
        else:
            identity, rj = x, j
        return F.conv_bn_act(out, self.conv3, self.bn3, "relu", residual=identity, residual_join=rj, residual_bn=rbn)


class _ResNetBase(tnn.Module):
    def _stem(self):
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)

    def forward(self, x):
        # conv -> BN -> ReLU -> maxpool: BN apply, ReLU and the pool run as one pass on the GPU
        # (the 112x112x64 BN output is never materialised; ops.bn._BNActPoolFn)
        x = F.conv_bn_act_maxpool(x, self.conv1, self.bn1, "relu", self.maxpool)
        x = self.conv2x(x)
        x = self.conv3x(x)
        x = self.conv4x(x)
        x = self.conv5x(x)
        x = self.avgpool(x)
        x = x.flatten(1)
        return self.linear(x)


class ResNet34(_ResNetBase):
    """Reference "ResNet-34": [2,2,2,2] BasicBlocks (= ResNet-18 depth)."""

    def __init__(self, num_classes=1000, layers=(2, 2, 2, 2)):
        super().__init__()
        self._stem()
        self.conv2x = self._make_blocks(layers[0], 64, 64, 1)
        self.conv3x = self._make_blocks(layers[1], 64, 128, 2)
        self.conv4x = self._make_blocks(layers[2], 128, 256, 2)
        self.conv5x = self._make_blocks(layers[3], 256, 512, 2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.linear = nn.Linear(512, num_classes)
        _init(self)

    @staticmethod
    def _make_blocks(n, cin, cout, stride):
        blocks = [BasicBlock(cin, cout, stride=stride, downsample=True)]
        blocks += [BasicBlock(cout, cout) for _ in range(1, n)]
        return nn.Sequential(*blocks)


class _Bottleneck(_ResNetBase):
    LAYERS = (3, 4, 6, 3)

    def __init__(self, num_classes=1000):
        super().__init__()
        self._stem()
        l1, l2, l3, l4 = self.LAYERS
        self.conv2x = self._make_blocks(l1, 64, 64, 256, 1)
        self.conv3x = self._make_blocks(l2, 256, 128, 512, 2)
        self.conv4x = self._make_blocks(l3, 512, 256, 1024, 2)
        self.conv5x = self._make_blocks(l4, 1024, 512, 2048, 2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.linear = nn.Linear(2048, num_classes)
        _init(self)

    @staticmethod
    def _make_blocks(n, cin, out1, out2, stride):
        blocks = [BottleneckBlock(cin, out1, out2, stride=stride, downsample=True)]
        blocks += [BottleneckBlock(out2, out1, out2) for _ in range(1, n)]
        return nn.Sequential(*blocks)


class ResNet50(_Bottleneck):
    LAYERS = (3, 4, 6, 3)


class ResNet152(_Bottleneck):
    LAYERS = (3, 8, 36, 3)
