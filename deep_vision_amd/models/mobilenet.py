"""MobileNet V1 (R/MobileNet/pytorch/models/mobilenet_v1.py:10-156) and its Keras variant
(R/MobileNet/tensorflow/models/mobilenet_v1.py:7-74), plus ShuffleNet V1 (the reference file
R/ShuffleNet/pytorch/models/shufflenet_v1.py is empty: built from the paper, g = 3).

MobileNet: depthwise 3x3 (groups = C) + BN + ReLU, pointwise 1x1 + BN + ReLU. On GPU the
depthwise runs the bandwidth-bound native stencil (csrc/depthwise.hip) with the BN statistics
fused into its epilogue, the pointwise runs the MFMA implicit GEMM.
The reference hard-codes BatchNorm2d(32) after the stem and multiplies channels by an integer
``alpha``; ``alpha`` may be any float here (channels rounded), alpha=1 is exact.
"""
from __future__ import annotations

import torch
import torch.nn as tnn

from .. import nn
from .. import ops as F
from ..ops.conv import no_wgrad_side


def _ch(c, alpha):
    return int(round(c * alpha))


class DepthwiseConv(tnn.Module):
    def __init__(self, in_channels, out_channels, stride):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, 3, padding=1, stride=stride, groups=in_channels, bias=False)
        self.bn = nn.BatchNorm2d(out_channels)
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        return F.conv_bn_act(x, self.conv, self.bn, "relu")


class PointwiseConv(tnn.Module):
    def __init__(self, in_channels, out_channels, stride):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, 1, stride=stride, bias=False)
        self.bn = nn.BatchNorm2d(out_channels)
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        return F.conv_bn_act(x, self.conv, self.bn, "relu")


class DepthwiseSeparableConv(tnn.Module):
    def __init__(self, in_channels, out_channels, dw_stride, pw_stride):
        super().__init__()
        self.dw = DepthwiseConv(in_channels, in_channels, stride=dw_stride)
        self.pw = PointwiseConv(in_channels, out_channels, stride=pw_stride)

    def forward(self, x):
        return self.pw(self.dw(x))


_MBV1_CFG = [(32, 64, 1), (64, 128, 2), (128, 128, 1), (128, 256, 2), (256, 256, 1), (256, 512, 2),
             (512, 512, 1), (512, 512, 1), (512, 512, 1), (512, 512, 1), (512, 512, 1), (512, 1024, 2),
             (1024, 1024, 1)]


class MobileNetV1(tnn.Module):
    def __init__(self, alpha=1, num_classes=1000):
        super().__init__()
        self.alpha = alpha
        c0 = _ch(32, alpha)
        layers = [nn.Conv2d(3, c0, 3, padding=1, stride=2, bias=False), nn.BatchNorm2d(c0), nn.ReLU(inplace=True)]
        for cin, cout, s in _MBV1_CFG:
            layers.append(DepthwiseSeparableConv(_ch(cin, alpha), _ch(cout, alpha), dw_stride=s, pw_stride=1))
        layers.append(nn.AdaptiveAvgPool2d((1, 1)))
        self.features = nn.FusedSequential(*layers)
        self.linear = nn.Linear(_ch(1024, alpha), num_classes)

    def forward(self, x):
        with no_wgrad_side():  # pointwise wgrads gain nothing on a side stream here (ops/conv.py WGRAD_SIDE)
            return self.linear(torch.flatten(self.features(x), 1))


class _SeparableConvTF(tnn.Module):
    """Keras SeparableConv block of the reference TF MobileNet: DepthwiseConv2D(+bias) -> BN ->
    ReLU -> 1x1 Conv2D(+bias) -> BN -> ReLU (R/MobileNet/tensorflow/models/mobilenet_v1.py:7-25)."""

    def __init__(self, cin, cout, stride):
        super().__init__()
        self.dw = nn.Conv2d(cin, cin, 3, stride=stride, padding=1, groups=cin, bias=True)
        self.bn1 = nn.BatchNorm2d(cin, eps=1e-3, momentum=0.01)
        self.pw = nn.Conv2d(cin, cout, 1, bias=True)
        self.bn2 = nn.BatchNorm2d(cout, eps=1e-3, momentum=0.01)

    def forward(self, x):
        x = F.conv_bn_act(x, self.dw, self.bn1, "relu")
        return F.conv_bn_act(x, self.pw, self.bn2, "relu")


class MobileNetV1TF(tnn.Module):
    """Keras MobileNet V1: first conv has no BN/ReLU (:32-37); AvgPool 7 then Dense — the
    reference applies Dense to a 4-D tensor; flattened here."""

    def __init__(self, num_classes=1000):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 32, 3, stride=2, padding=1)
        self.blocks = tnn.Sequential(*[_SeparableConvTF(ci, co, s) for ci, co, s in _MBV1_CFG])
        self.pool = nn.AvgPool2d(7)
        self.fc = nn.Linear(1024, num_classes)

    def forward(self, x):
        with no_wgrad_side():
            x = self.blocks(self.conv1(x))
            return self.fc(torch.flatten(self.pool(x), 1))


# ------------------------------------ ShuffleNet V1 ------------------------------------
class ShuffleUnit(tnn.Module):
    """ShuffleNet V1 unit (Zhang et al. 2017, Fig. 2b/c): grouped 1x1 -> BN -> ReLU -> channel
    shuffle -> depthwise 3x3 (stride) -> BN -> grouped 1x1 -> BN, residual add (stride 1) or
    concat with a 3x3/2 average-pooled shortcut (stride 2), ReLU.

    The shuffle is applied right after the first grouped 1x1 (conv -> shuffle -> BN -> ReLU):
    BN and ReLU act per channel, so this is the paper's block with bn1's parameters indexed in the
    shuffled channel order, and it lets the shuffle ride on the grouped conv's store
    (csrc/gconv.hip) instead of a separate pass. The torch path runs the same order."""

    def __init__(self, cin, cout, groups, stride, first_group=True):
        super().__init__()
        self.stride = stride
        mid = cout // 4
        out = cout - cin if stride == 2 else cout
        g1 = groups if first_group else 1
        self.gconv1 = nn.Conv2d(cin, mid, 1, groups=g1, bias=False)
        self.bn1 = nn.BatchNorm2d(mid)
        self.groups = groups
        self.dwconv = nn.Conv2d(mid, mid, 3, stride=stride, padding=1, groups=mid, bias=False)
        self.bn2 = nn.BatchNorm2d(mid)
        self.gconv2 = nn.Conv2d(mid, out, 1, groups=groups, bias=False)
        self.bn3 = nn.BatchNorm2d(out)

    def forward(self, x):
        y = F.conv_bn_act(x, self.gconv1, self.bn1, "relu", shuffle=self.groups)
        y = F.conv_bn_act(y, self.dwconv, self.bn2, None)
        if self.stride == 1:
            return F.conv_bn_act(y, self.gconv2, self.bn3, "relu", residual=x)
        y = F.conv_bn_act(y, self.gconv2, self.bn3, None)
        sc = F.avg_pool2d(x, 3, 2, 1)
        return F.relu(F.concat([sc, y]))


class ShuffleNetV1(tnn.Module):
    """ShuffleNet V1 1x, g = 3 (paper Table 1): 24 -> 240 -> 480 -> 960 channels."""

    STAGE_OUT = {1: (144, 288, 576), 2: (200, 400, 800), 3: (240, 480, 960), 4: (272, 544, 1088), 8: (384, 768, 1536)}

    def __init__(self, groups=3, num_classes=1000, stage_repeats=(3, 7, 3)):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 24, 3, stride=2, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(24)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        stages, cin = [], 24
        for si, (cout, rep) in enumerate(zip(self.STAGE_OUT[groups], stage_repeats)):
            units = [ShuffleUnit(cin, cout, groups, 2, first_group=si > 0)]
            units += [ShuffleUnit(cout, cout, groups, 1) for _ in range(rep)]
            stages.append(tnn.Sequential(*units))
            cin = cout
        self.stage2, self.stage3, self.stage4 = stages
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(cin, num_classes)

    def forward(self, x):
        x = F.conv_bn_act(x, self.conv1, self.bn1, "relu")
        x = self.maxpool(x)
        x = self.stage4(self.stage3(self.stage2(x)))
        return self.fc(torch.flatten(self.avgpool(x), 1))
