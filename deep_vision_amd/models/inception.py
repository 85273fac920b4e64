"""Inception V1 / GoogLeNet with the reference topology (R/Inception/pytorch/models/inception_v1.py:9-200):
conv+ReLU ``BasicConv2d`` units, ceil-mode max pools, LRN with size = channels, four-branch
modules concatenated on channels, two auxiliary heads active in training mode.

Train mode returns ``(out, aux1, aux2)`` (reference :112-113); the trainer combines them as
CE(out) + 0.3*(CE(aux1)+CE(aux2)) (GoogLeNet paper), fixing SURVEY Appendix A3.

``InceptionV3`` is a stub in the reference (R/Inception/pytorch/models/inception_v3.py:1-6,
README "WIP"); a full Inception V3 is provided here as an extension (torchvision topology).
"""
from __future__ import annotations

import torch
import torch.nn as tnn

from .. import nn
from .. import ops as F


class BasicConv2d(tnn.Module):
    def __init__(self, in_channels, out_channels, kernel_size, **kw):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size, **kw)

    def forward(self, x, out=None):
        c = self.conv
        return F.conv2d(x, c.weight, c.bias, c.stride, c.padding, c.dilation, c.groups, act="relu", out=out)


class InceptionModule(tnn.Module):
    def __init__(self, in_channels, p1, p2, p3, p4, p5, p6):
        super().__init__()
        self.branch1_conv1x1 = BasicConv2d(in_channels, p1, 1, stride=1)
        self.branch2_conv1x1 = BasicConv2d(in_channels, p2, 1, stride=1)
        self.branch2_conv3x3 = BasicConv2d(p2, p3, 3, stride=1, padding=1)
        self.branch3_conv1x1 = BasicConv2d(in_channels, p4, 1, stride=1)
        self.branch3_conv5x5 = BasicConv2d(p4, p5, 5, stride=1, padding=2)
        self.branch4_maxpool = nn.MaxPool2d(3, 1, padding=1)
        self.branch4_conv1x1 = BasicConv2d(in_channels, p6, 1, stride=1)

    def forward(self, x):
        outs = [None] * 4
        if F.native(x):
            # write-into-slice concat: each branch's last conv epilogue stores straight into its
            # channel slice of the module output (R/Inception/pytorch/models/inception_v1.py:156-158)
            N, _, H, W = x.shape
            outs = F.concat_slices(N, [m.conv.out_channels for m in self._last()], H, W, x.device)
        b1 = self.branch1_conv1x1(x, out=outs[0])
        b2 = self.branch2_conv3x3(self.branch2_conv1x1(x), out=outs[1])
        b3 = self.branch3_conv5x5(self.branch3_conv1x1(x), out=outs[2])
        b4 = self.branch4_conv1x1(self.branch4_maxpool(x), out=outs[3])
        if F.native(x):
            return F.slice_cat([b1, b2, b3, b4])
        return torch.cat([b1, b2, b3, b4], 1)

    def _last(self):
        return (self.branch1_conv1x1, self.branch2_conv3x3, self.branch3_conv5x5, self.branch4_conv1x1)


class AuxiliaryClassifier(tnn.Module):
    def __init__(self, in_channels, num_classes=1000):
        super().__init__()
        self.features = tnn.Sequential(nn.AvgPool2d(5, 3), BasicConv2d(in_channels, 128, 1))
        self.classifier = nn.FusedSequential(
            nn.Linear(4 * 4 * 128, 1024), nn.ReLU(inplace=True), nn.Dropout(p=0.7), nn.Linear(1024, num_classes))

    def forward(self, x):
        return self.classifier(torch.flatten(self.features(x), 1))


class InceptionV1(tnn.Module):
    def __init__(self, num_classes=1000, aux_logits=True):
        super().__init__()
        self.conv7x7 = BasicConv2d(3, 64, 7, stride=2, padding=3)
        self.maxpool1 = nn.MaxPool2d(3, 2, ceil_mode=True)
        self.lrn1 = nn.LocalResponseNorm(64)
        self.conv1x1 = BasicConv2d(64, 64, 1, stride=1)
        self.conv3x3 = BasicConv2d(64, 192, 3, stride=1, padding=1)
        self.maxpool2 = nn.MaxPool2d(3, 2, ceil_mode=True)
        self.lrn2 = nn.LocalResponseNorm(192)
        self.inception_3a = InceptionModule(192, 64, 96, 128, 16, 32, 32)
        self.inception_3b = InceptionModule(256, 128, 128, 192, 32, 96, 64)
        self.maxpool3 = nn.MaxPool2d(3, 2, ceil_mode=True)
        self.inception_4a = InceptionModule(480, 192, 96, 208, 16, 48, 64)
        self.aux1 = AuxiliaryClassifier(512, num_classes) if aux_logits else None
        self.inception_4b = InceptionModule(512, 160, 112, 224, 24, 64, 64)
        self.inception_4c = InceptionModule(512, 128, 128, 256, 24, 64, 64)
        self.inception_4d = InceptionModule(512, 112, 144, 288, 32, 64, 64)
        self.aux2 = AuxiliaryClassifier(528, num_classes) if aux_logits else None
        self.inception_4e = InceptionModule(528, 256, 160, 320, 32, 128, 128)
        self.maxpool4 = nn.MaxPool2d(3, 2, ceil_mode=True)
        self.inception_5a = InceptionModule(832, 256, 160, 320, 32, 128, 128)
        self.inception_5b = InceptionModule(832, 384, 192, 384, 48, 128, 128)
        self.avgpool = nn.AvgPool2d(7, stride=1)
        self.dropout = nn.Dropout(p=0.4)
        self.linear = nn.Linear(1024, num_classes)
        for m in self.modules():  # R/Inception/pytorch/models/inception_v1.py:117-127
            if isinstance(m, tnn.Conv2d):
                tnn.init.xavier_normal_(m.weight)
                if m.bias is not None:
                    tnn.init.constant_(m.bias, 0)
            elif isinstance(m, tnn.Linear):
                tnn.init.normal_(m.weight, 0, 0.01)
                tnn.init.constant_(m.bias, 0)

    def forward(self, x):
        x = self.conv7x7(x)
        x = self.maxpool1(x)
        x = self.lrn1(x)
        x = self.conv1x1(x)
        x = self.conv3x3(x)
        x = self.lrn2(x)
        x = self.maxpool2(x)
        x = self.inception_3a(x)
        x = self.inception_3b(x)
        x = self.maxpool3(x)
        x = self.inception_4a(x)
        aux1 = self.aux1(x) if (self.training and self.aux1 is not None) else None
        x = self.inception_4b(x)
        x = self.inception_4c(x)
        x = self.inception_4d(x)
        aux2 = self.aux2(x) if (self.training and self.aux2 is not None) else None
        x = self.inception_4e(x)
        x = self.maxpool4(x)
        x = self.inception_5a(x)
        x = self.inception_5b(x)
        x = self.avgpool(x)
        x = self.dropout(torch.flatten(x, 1))
        out = self.linear(x)
        if aux1 is not None and aux2 is not None:
            return out, aux1, aux2
        return out


# ------------------------------ Inception V3 (extension) ------------------------------
class _CBR(tnn.Module):
    def __init__(self, cin, cout, k, **kw):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, k, bias=False, **kw)
        self.bn = nn.BatchNorm2d(cout, eps=0.001)

    def forward(self, x):
        return F.conv_bn_act(x, self.conv, self.bn, "relu")


def _cat(xs, ref):
    return F.concat(xs)  # native slice copies on the GPU path


class _InceptionA(tnn.Module):
    def __init__(self, cin, pool_features):
        super().__init__()
        self.branch1x1 = _CBR(cin, 64, 1)
        self.branch5x5_1 = _CBR(cin, 48, 1)
        self.branch5x5_2 = _CBR(48, 64, 5, padding=2)
        self.branch3x3dbl_1 = _CBR(cin, 64, 1)
        self.branch3x3dbl_2 = _CBR(64, 96, 3, padding=1)
        self.branch3x3dbl_3 = _CBR(96, 96, 3, padding=1)
        self.branch_pool = _CBR(cin, pool_features, 1)

    def forward(self, x):
        b1 = self.branch1x1(x)
        b5 = self.branch5x5_2(self.branch5x5_1(x))
        b3 = self.branch3x3dbl_3(self.branch3x3dbl_2(self.branch3x3dbl_1(x)))
        bp = self.branch_pool(F.avg_pool2d(x, 3, 1, 1))
        return _cat([b1, b5, b3, bp], x)


class _InceptionB(tnn.Module):
    def __init__(self, cin):
        super().__init__()
        self.branch3x3 = _CBR(cin, 384, 3, stride=2)
        self.branch3x3dbl_1 = _CBR(cin, 64, 1)
        self.branch3x3dbl_2 = _CBR(64, 96, 3, padding=1)
        self.branch3x3dbl_3 = _CBR(96, 96, 3, stride=2)

    def forward(self, x):
        b3 = self.branch3x3(x)
        bd = self.branch3x3dbl_3(self.branch3x3dbl_2(self.branch3x3dbl_1(x)))
        return _cat([b3, bd, F.max_pool2d(x, 3, 2)], x)


class _InceptionC(tnn.Module):
    def __init__(self, cin, c7):
        super().__init__()
        self.branch1x1 = _CBR(cin, 192, 1)
        self.branch7x7_1 = _CBR(cin, c7, 1)
        self.branch7x7_2 = _CBR(c7, c7, (1, 7), padding=(0, 3))
        self.branch7x7_3 = _CBR(c7, 192, (7, 1), padding=(3, 0))
        self.branch7x7dbl_1 = _CBR(cin, c7, 1)
        self.branch7x7dbl_2 = _CBR(c7, c7, (7, 1), padding=(3, 0))
        self.branch7x7dbl_3 = _CBR(c7, c7, (1, 7), padding=(0, 3))
        self.branch7x7dbl_4 = _CBR(c7, c7, (7, 1), padding=(3, 0))
        self.branch7x7dbl_5 = _CBR(c7, 192, (1, 7), padding=(0, 3))
        self.branch_pool = _CBR(cin, 192, 1)

    def forward(self, x):
        b1 = self.branch1x1(x)
        b7 = self.branch7x7_3(self.branch7x7_2(self.branch7x7_1(x)))
        bd = x
        for m in (self.branch7x7dbl_1, self.branch7x7dbl_2, self.branch7x7dbl_3, self.branch7x7dbl_4,
                  self.branch7x7dbl_5):
            bd = m(bd)
        bp = self.branch_pool(F.avg_pool2d(x, 3, 1, 1))
        return _cat([b1, b7, bd, bp], x)


class _InceptionD(tnn.Module):
    def __init__(self, cin):
        super().__init__()
        self.branch3x3_1 = _CBR(cin, 192, 1)
        self.branch3x3_2 = _CBR(192, 320, 3, stride=2)
        self.branch7x7x3_1 = _CBR(cin, 192, 1)
        self.branch7x7x3_2 = _CBR(192, 192, (1, 7), padding=(0, 3))
        self.branch7x7x3_3 = _CBR(192, 192, (7, 1), padding=(3, 0))
        self.branch7x7x3_4 = _CBR(192, 192, 3, stride=2)

    def forward(self, x):
        b3 = self.branch3x3_2(self.branch3x3_1(x))
        b7 = self.branch7x7x3_4(self.branch7x7x3_3(self.branch7x7x3_2(self.branch7x7x3_1(x))))
        return _cat([b3, b7, F.max_pool2d(x, 3, 2)], x)


class _InceptionE(tnn.Module):
    def __init__(self, cin):
        super().__init__()
        self.branch1x1 = _CBR(cin, 320, 1)
        self.branch3x3_1 = _CBR(cin, 384, 1)
        self.branch3x3_2a = _CBR(384, 384, (1, 3), padding=(0, 1))
        self.branch3x3_2b = _CBR(384, 384, (3, 1), padding=(1, 0))
        self.branch3x3dbl_1 = _CBR(cin, 448, 1)
        self.branch3x3dbl_2 = _CBR(448, 384, 3, padding=1)
        self.branch3x3dbl_3a = _CBR(384, 384, (1, 3), padding=(0, 1))
        self.branch3x3dbl_3b = _CBR(384, 384, (3, 1), padding=(1, 0))
        self.branch_pool = _CBR(cin, 192, 1)

    def forward(self, x):
        b1 = self.branch1x1(x)
        t = self.branch3x3_1(x)
        b3 = _cat([self.branch3x3_2a(t), self.branch3x3_2b(t)], x)
        t = self.branch3x3dbl_2(self.branch3x3dbl_1(x))
        bd = _cat([self.branch3x3dbl_3a(t), self.branch3x3dbl_3b(t)], x)
        bp = self.branch_pool(F.avg_pool2d(x, 3, 1, 1))
        return _cat([b1, b3, bd, bp], x)


class InceptionV3(tnn.Module):
    """Inception V3 (299x299 input). Extension: the reference file is an empty stub."""

    def __init__(self, num_classes=1000):
        super().__init__()
        self.Conv2d_1a_3x3 = _CBR(3, 32, 3, stride=2)
        self.Conv2d_2a_3x3 = _CBR(32, 32, 3)
        self.Conv2d_2b_3x3 = _CBR(32, 64, 3, padding=1)
        self.Conv2d_3b_1x1 = _CBR(64, 80, 1)
        self.Conv2d_4a_3x3 = _CBR(80, 192, 3)
        self.Mixed_5b = _InceptionA(192, 32)
        self.Mixed_5c = _InceptionA(256, 64)
        self.Mixed_5d = _InceptionA(288, 64)
        self.Mixed_6a = _InceptionB(288)
        self.Mixed_6b = _InceptionC(768, 128)
        self.Mixed_6c = _InceptionC(768, 160)
        self.Mixed_6d = _InceptionC(768, 160)
        self.Mixed_6e = _InceptionC(768, 192)
        self.Mixed_7a = _InceptionD(768)
        self.Mixed_7b = _InceptionE(1280)
        self.Mixed_7c = _InceptionE(2048)
        self.dropout = nn.Dropout(0.5)
        self.fc = nn.Linear(2048, num_classes)

    def forward(self, x):
        x = self.Conv2d_2b_3x3(self.Conv2d_2a_3x3(self.Conv2d_1a_3x3(x)))
        x = F.max_pool2d(x, 3, 2)
        x = self.Conv2d_4a_3x3(self.Conv2d_3b_1x1(x))
        x = F.max_pool2d(x, 3, 2)
        for m in (self.Mixed_5b, self.Mixed_5c, self.Mixed_5d, self.Mixed_6a, self.Mixed_6b, self.Mixed_6c,
                  self.Mixed_6d, self.Mixed_6e, self.Mixed_7a, self.Mixed_7b, self.Mixed_7c):
            x = m(x)
        x = F.adaptive_avg_pool2d(x, 1)
        return self.fc(self.dropout(torch.flatten(x, 1)))
