"""CenterNet / "Objects as Points" with a 2-stack order-5 hourglass (R/ObjectsAsPoints/tensorflow/model.py:17-179).

* ResidualBlock: 1x1 (stride s) conv -> BN -> ReLU -> 3x3 conv -> BN, + identity (or 1x1/s conv -> BN
  projection when the width or stride changes), ReLU (:35-69). Convs have no bias; Keras BN
  (eps 1e-3, momentum .99 -> torch .01).
* HourglassModule(order): filters / residual counts per order from ``order_to_filters`` /
  ``order_to_num_residual`` (:17-32); the down path is a stride-2 residual block (:94-127).
* ObjectsAsPoints: 7x7/2 stem (128) -> stride-2 residual (256) -> 2 x [hourglass -> 3x3 conv+BN+ReLU
  -> heads (heatmap C, size 2, offset 2: 3x3 conv(256)+ReLU -> 3x3 conv)] (:130-179).

Reference quirks kept: the ``low3`` loop result is discarded (:118-121) and the
``intermediate`` merge of the two stacks is overwritten by ``ResidualBlock(x)`` (:170-176). Those
layers never reach an output, so the Keras functional Model leaves them out; they are not built
here either, which reproduces the reference's recorded summary exactly (94,654,504 total /
94,553,384 trainable, R/ObjectsAsPoints/tensorflow/test.ipynb cell 2; pinned in tests).
"""
from __future__ import annotations

import torch.nn as tnn

from .. import nn
from .. import ops as F

ORDER_TO_FILTERS = {5: (256, 256), 4: (256, 384), 3: (384, 384), 2: (384, 384), 1: (384, 512)}
ORDER_TO_NUM_RESIDUAL = {5: (2, 2), 4: (2, 2), 3: (2, 2), 2: (2, 2), 1: (2, 4)}


def _bn(c):
    return nn.BatchNorm2d(c, eps=1e-3, momentum=0.01)


def _conv(cin, cout, k, stride=1, bias=False):
    return nn.Conv2d(cin, cout, k, stride=stride, padding="same_keras", bias=bias)


class ResidualBlock(tnn.Module):
    def __init__(self, cin, cout, stride=1):
        super().__init__()
        self.proj = None
        if cin != cout or stride > 1:
            self.proj = tnn.ModuleDict({"conv": _conv(cin, cout, 1, stride), "bn": _bn(cout)})
        self.conv1 = _conv(cin, cout, 1, stride)
        self.bn1 = _bn(cout)
        self.conv2 = _conv(cout, cout, 3)
        self.bn2 = _bn(cout)

    def forward(self, x):
        identity = x if self.proj is None else F.conv_bn_act(x, self.proj["conv"], self.proj["bn"])
        y = F.conv_bn_act(x, self.conv1, self.bn1, "relu")
        return F.conv_bn_act(y, self.conv2, self.bn2, "relu", residual=identity)


class HourglassModule(tnn.Module):
    def __init__(self, order):
        super().__init__()
        cur, nxt = ORDER_TO_FILTERS[order]
        cur_r, nxt_r = ORDER_TO_NUM_RESIDUAL[order]
        self.up1 = tnn.Sequential(*[ResidualBlock(cur, cur) for _ in range(cur_r)])
        self.low1 = tnn.Sequential(ResidualBlock(cur, nxt, stride=2),
                                   *[ResidualBlock(nxt, nxt) for _ in range(cur_r - 1)])
        if order > 1:
            self.low2 = HourglassModule(order - 1)
        else:
            self.low2 = tnn.Sequential(*[ResidualBlock(nxt, nxt) for _ in range(nxt_r)])
        self.low3 = ResidualBlock(nxt, cur)

    def forward(self, x):
        up1 = self.up1(x)
        low2 = self.low2(self.low1(x))
        return F.add(up1, F.upsample_nearest(self.low3(low2), 2))


class DetectionConv(tnn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.conv1 = _conv(cin, 256, 3, bias=True)
        self.conv2 = _conv(256, cout, 3, bias=True)

    def forward(self, x):
        return self.conv2(F.conv2d(x, self.conv1.weight, self.conv1.bias, 1, 1, act="relu"))


class ObjectsAsPoints(tnn.Module):
    def __init__(self, num_stack=2, num_classes=80, input_size=256):
        super().__init__()
        self.num_stack = num_stack
        self.num_classes = num_classes
        self.input_size = input_size
        self.stem = _conv(3, 128, 7, 2)
        self.stem_bn = _bn(128)
        self.pre = ResidualBlock(128, 256, stride=2)
        self.hourglass = tnn.ModuleList(HourglassModule(5) for _ in range(num_stack))
        self.cnv = tnn.ModuleList(tnn.ModuleDict({"conv": _conv(256, 256, 3, bias=True), "bn": _bn(256)})
                                  for _ in range(num_stack))
        self.heads = tnn.ModuleList(tnn.ModuleDict({"heatmap": DetectionConv(256, num_classes),
                                                    "size": DetectionConv(256, 2), "offset": DetectionConv(256, 2)})
                                    for _ in range(num_stack))
        # input of stack i+1 = ResidualBlock(x) (:176; the x1/x2 merge above it is dead)
        self.merge = tnn.ModuleList(ResidualBlock(256, 256) for _ in range(num_stack - 1))

    def forward(self, x):
        """List over stacks of (heatmap logits (N, C, g, g), size (N, 2, g, g), offset (N, 2, g, g))."""
        x = F.conv_bn_act(x, self.stem, self.stem_bn, "relu")
        inter = self.pre(x)
        ys = []
        for i in range(self.num_stack):
            x = self.hourglass[i](inter)
            c = self.cnv[i]
            x = F.conv_bn_act(x, c["conv"], c["bn"], "relu")
            h = self.heads[i]
            ys.append((h["heatmap"](x), h["size"](x), h["offset"](x)))
            if i < self.num_stack - 1:
                inter = self.merge[i](x)
        return ys
