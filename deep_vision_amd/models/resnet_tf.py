"""Keras-origin ResNets of the reference (R/ResNet/tensorflow/models/).

* ResNet50TF / ResNet152TF (resnet50.py:9-120, resnet152.py): ZeroPadding(3) + 7x7/2 valid conv
  (no bias) -> BN -> ReLU -> 3x3/2 max-pool *without* padding; bottleneck V1 with the stride on
  the first 1x1, a projection (1x1 conv + BN) on the first block of each stage, and **no BN
  after the last 1x1** before the add -> ReLU. Keras BN eps 1e-3 / momentum .99.
  The Keras ``kernel_regularizer=l2(1e-4)`` is expressed as optimizer weight decay (2e-4 on
  the conv kernels, config ``tf_resnet50``).
* ResNet50V2 (resnet50v2.py): pre-activation bottlenecks, stride on the *last* block of a
  stage (identity = 1x1 max-pool subsample), 3x3 conv padded explicitly then 'valid',
  post BN + ReLU, GAP, Dense. ``pretrain`` weights (a download) are not available offline.
All output logits (the Keras heads end in softmax; the loss applies log-softmax).
"""
from __future__ import annotations

import torch
import torch.nn as tnn

from .. import nn
from .. import ops as F


def _bn(c):
    return nn.BatchNorm2d(c, eps=1e-3, momentum=0.01)


def _he(m):
    for mod in m.modules():
        if isinstance(mod, tnn.Conv2d):
            tnn.init.kaiming_normal_(mod.weight, mode="fan_in", nonlinearity="relu")


class BottleneckTF(tnn.Module):
    def __init__(self, cin, c1, c2, stride=1, downsample=False):
        super().__init__()
        self.proj = tnn.ModuleDict({"conv": nn.Conv2d(cin, c2, 1, stride=stride, bias=False), "bn": _bn(c2)}) \
            if downsample else None
        self.conv1 = nn.Conv2d(cin, c1, 1, stride=stride, bias=False)
        self.bn1 = _bn(c1)
        self.conv2 = nn.Conv2d(c1, c1, 3, padding=1, bias=False)
        self.bn2 = _bn(c1)
        self.conv3 = nn.Conv2d(c1, c2, 1, bias=False)

    def forward(self, x):
        idn = F.conv_bn_act(x, self.proj["conv"], self.proj["bn"]) if self.proj is not None else x
        y = F.conv_bn_act(x, self.conv1, self.bn1, "relu")
        y = F.conv_bn_act(y, self.conv2, self.bn2, "relu")
        return F.add(self.conv3(y), idn, act="relu")


class _ResNetTF(tnn.Module):
    BLOCKS = (3, 4, 6, 3)

    def __init__(self, num_classes=1000):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = _bn(64)
        stages, cin = [], 64
        for i, (n, c1) in enumerate(zip(self.BLOCKS, (64, 128, 256, 512))):
            c2 = 4 * c1
            blocks = [BottleneckTF(cin, c1, c2, stride=1 if i == 0 else 2, downsample=True)]
            blocks += [BottleneckTF(c2, c1, c2) for _ in range(n - 1)]
            stages.append(tnn.Sequential(*blocks))
            cin = c2
        self.stages = tnn.Sequential(*stages)
        self.fc = nn.Linear(2048, num_classes)
        _he(self)

    def forward(self, x):
        x = F.conv_bn_act(x, self.conv1, self.bn1, "relu")
        x = F.max_pool2d(x, 3, 2)
        x = self.stages(x)
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


class ResNet50TF(_ResNetTF):
    BLOCKS = (3, 4, 6, 3)


class ResNet152TF(_ResNetTF):
    BLOCKS = (3, 8, 36, 3)


class BottleneckV2(tnn.Module):
    def __init__(self, cin, f, stride=1, downsample=False):
        super().__init__()
        self.stride = stride
        self.preact_bn = _bn(cin)
        self.conv0 = nn.Conv2d(cin, 4 * f, 1, stride=stride) if downsample else None
        self.conv1 = nn.Conv2d(cin, f, 1, bias=False)
        self.bn1 = _bn(f)
        self.conv2 = nn.Conv2d(f, f, 3, stride=stride, padding=1, bias=False)
        self.bn2 = _bn(f)
        self.conv3 = nn.Conv2d(f, 4 * f, 1)

    def forward(self, x):
        pre = F.batch_norm_act(x, self.preact_bn, "relu")
        if self.conv0 is not None:
            idn = self.conv0(pre)
        elif self.stride > 1:
            idn = x[:, :, ::self.stride, ::self.stride]  # MaxPooling2D(1, strides)
            if F.native(x):
                idn = idn.contiguous(memory_format=torch.channels_last)
        else:
            idn = x
        y = F.conv_bn_act(pre, self.conv1, self.bn1, "relu")
        y = F.conv_bn_act(y, self.conv2, self.bn2, "relu")
        return F.add(self.conv3(y), idn)


class ResNet50V2(tnn.Module):
    def __init__(self, num_classes=1000):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3)
        blocks, cin = [], 64
        for n, f, s in ((3, 64, 2), (4, 128, 2), (6, 256, 2), (3, 512, 1)):
            blocks.append(BottleneckV2(cin, f, downsample=True))
            blocks += [BottleneckV2(4 * f, f) for _ in range(n - 2)]
            blocks.append(BottleneckV2(4 * f, f, stride=s))
            cin = 4 * f
        self.blocks = tnn.Sequential(*blocks)
        self.post_bn = _bn(2048)
        self.fc = nn.Linear(2048, num_classes)
        _he(self)

    def forward(self, x):
        x = F.max_pool2d(self.conv1(x), 3, 2, 1)
        x = F.batch_norm_act(self.blocks(x), self.post_bn, "relu")
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))
