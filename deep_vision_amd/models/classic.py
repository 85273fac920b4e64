"""LeNet-5, AlexNet V1/V2 and VGG-16/19 with the reference's exact topology, parameter names
and initialisation (parameter counts pinned in tests/test_models.py against SURVEY §2.2).

* LeNet5        R/LeNet/pytorch/models/lenet5.py:8-67        (tanh after every pool)
* LeNet5TF      R/LeNet/tensorflow/models/lenet5.py:7-34     (sigmoid after the pools, A20)
* AlexNetV1     R/AlexNet/pytorch/models/alexnet_v1.py:11-125 (one tower, LRN size = C, A4)
* AlexNetV2     R/AlexNet/pytorch/models/alexnet_v2.py:12-75
* AlexNetV2TF   R/AlexNet/tensorflow/models/alexnet_v2.py:25-70 (ZeroPad 3, valid conv, TF LRN)
* VGG16 / VGG19 R/VGG/pytorch/models/vgg16.py:8-127 / vgg19.py (Xavier conv, N(0, .01) linear)

``FusedSequential`` keeps nn.Sequential indices (state_dict keys) while fusing conv+bias+ReLU
and Linear+ReLU into single native kernels on GPU.
"""
from __future__ import annotations

import torch
import torch.nn as tnn

from .. import nn
from .. import ops as F
from ..ops.lrn import tf_local_response_norm


class LeNet5(tnn.Module):
    def __init__(self, num_classes=10):
        super().__init__()
        self.features = nn.FusedSequential(
            nn.Conv2d(1, 6, 5, stride=1), nn.Tanh(), nn.AvgPool2d(2, stride=2), nn.Tanh(),
            nn.Conv2d(6, 16, 5, stride=1), nn.Tanh(), nn.AvgPool2d(2, stride=2), nn.Tanh(),
            nn.Conv2d(16, 120, 5), nn.Tanh(),
        )
        self.classifier = nn.FusedSequential(nn.Linear(120, 84), nn.Tanh(), nn.Linear(84, num_classes))

    def forward(self, x):
        x = self.features(x)
        return self.classifier(torch.flatten(x, 1))


class LeNet5TF(tnn.Module):
    """Keras LeNet-5 (R/LeNet/tensorflow/models/lenet5.py): tanh convs, avgpool + sigmoid,
    dense tanh, softmax head (logits here; the loss applies log-softmax)."""

    def __init__(self, num_classes=10):
        super().__init__()
        self.features = nn.FusedSequential(
            nn.Conv2d(1, 6, 5), nn.Tanh(), nn.AvgPool2d(2, 2), nn.Sigmoid(),
            nn.Conv2d(6, 16, 5), nn.Tanh(), nn.AvgPool2d(2, 2), nn.Sigmoid(),
            nn.Conv2d(16, 120, 5), nn.Tanh(),
        )
        self.classifier = nn.FusedSequential(nn.Linear(120, 84), nn.Tanh(), nn.Linear(84, num_classes))

    def forward(self, x):
        return self.classifier(torch.flatten(self.features(x), 1))


def _alexnet_classifier(num_classes):
    return nn.FusedSequential(
        nn.Dropout(p=0.5), nn.Linear(6 * 6 * 256, 4096), nn.ReLU(inplace=True),
        nn.Dropout(p=0.5), nn.Linear(4096, 4096), nn.ReLU(inplace=True),
        nn.Linear(4096, num_classes),
    )


class AlexNetV1(tnn.Module):
    def __init__(self, num_classes=1000):
        super().__init__()
        self.features = nn.FusedSequential(
            nn.Conv2d(3, 96, 11, stride=4, padding=2), nn.ReLU(inplace=True), nn.LocalResponseNorm(96),
            nn.MaxPool2d(3, 2),
            nn.Conv2d(96, 256, 5, stride=1, padding=2), nn.ReLU(inplace=True), nn.LocalResponseNorm(256),
            nn.MaxPool2d(3, 2),
            nn.Conv2d(256, 384, 3, stride=1, padding=1), nn.ReLU(inplace=True),
            nn.Conv2d(384, 384, 3, stride=1, padding=1), nn.ReLU(inplace=True),
            nn.Conv2d(384, 256, 3, stride=1, padding=1), nn.ReLU(inplace=True),
            nn.MaxPool2d(3, 2),
        )
        self.classifier = _alexnet_classifier(num_classes)

    def forward(self, x):
        return self.classifier(torch.flatten(self.features(x), 1))


class AlexNetV2(tnn.Module):
    def __init__(self, num_classes=1000):
        super().__init__()
        self.features = nn.FusedSequential(
            nn.Conv2d(3, 64, 11, stride=4, padding=2), nn.ReLU(inplace=True), nn.LocalResponseNorm(64),
            nn.MaxPool2d(3, 2),
            nn.Conv2d(64, 192, 5, stride=1, padding=2), nn.ReLU(inplace=True), nn.LocalResponseNorm(192),
            nn.MaxPool2d(3, 2),
            nn.Conv2d(192, 384, 3, stride=1, padding=1), nn.ReLU(inplace=True),
            nn.Conv2d(384, 384, 3, stride=1, padding=1), nn.ReLU(inplace=True),
            nn.Conv2d(384, 256, 3, stride=1, padding=1), nn.ReLU(inplace=True),
            nn.MaxPool2d(3, 2),
        )
        self.classifier = _alexnet_classifier(num_classes)

    def forward(self, x):
        return self.classifier(torch.flatten(self.features(x), 1))


class _TFLRN(tnn.Module):
    """tf.nn.local_response_normalization defaults (depth_radius 5, bias 1, alpha 1, beta .5)."""

    def __init__(self, depth_radius=5, bias=1.0, alpha=1.0, beta=0.5):
        super().__init__()
        self.r, self.b, self.a, self.beta = depth_radius, bias, alpha, beta

    def forward(self, x):
        return tf_local_response_norm(x, self.r, self.b, self.a, self.beta)


class AlexNetV2TF(tnn.Module):
    """Keras AlexNet V2 (R/AlexNet/tensorflow/models/alexnet_v2.py:25-70): ZeroPadding2D(3) to 230,
    valid 11x11/4 conv, custom LRN layer with TF defaults, maxpool 3/2, dense 4096 x2."""

    def __init__(self, num_classes=1000):
        super().__init__()
        self.features = nn.FusedSequential(
            nn.ZeroPad2d(3),
            nn.Conv2d(3, 64, 11, stride=4), nn.ReLU(), _TFLRN(), nn.MaxPool2d(3, 2),
            nn.Conv2d(64, 192, 5, padding=2), nn.ReLU(), _TFLRN(), nn.MaxPool2d(3, 2),
            nn.Conv2d(192, 384, 3, padding=1), nn.ReLU(),
            nn.Conv2d(384, 384, 3, padding=1), nn.ReLU(),
            nn.Conv2d(384, 256, 3, padding=1), nn.ReLU(), nn.MaxPool2d(3, 2),
        )
        self.classifier = _alexnet_classifier(num_classes)

    def forward(self, x):
        return self.classifier(torch.flatten(self.features(x), 1))


def _vgg_features(cfg):
    layers, cin = [], 3
    for v in cfg:
        if v == "M":
            layers.append(nn.MaxPool2d(2, 2))
        else:
            layers += [nn.Conv2d(cin, v, 3, stride=1, padding=1), nn.ReLU(inplace=True)]
            cin = v
    return nn.FusedSequential(*layers)


class _VGG(tnn.Module):
    CFG: list = []

    def __init__(self, num_classes=1000):
        super().__init__()
        self.features = _vgg_features(self.CFG)
        self.classifier = nn.FusedSequential(
            nn.Dropout(p=0.5), nn.Linear(7 * 7 * 512, 4096), nn.ReLU(inplace=True),
            nn.Dropout(p=0.5), nn.Linear(4096, 4096), nn.ReLU(inplace=True),
            nn.Linear(4096, num_classes),
        )
        # R/VGG/pytorch/models/vgg16.py:112-127
        for m in self.modules():
            if isinstance(m, tnn.Conv2d):
                tnn.init.xavier_normal_(m.weight)
                if m.bias is not None:
                    tnn.init.constant_(m.bias, 0)
            elif isinstance(m, tnn.Linear):
                tnn.init.normal_(m.weight, 0, 0.01)
                tnn.init.constant_(m.bias, 0)

    def forward(self, x):
        return self.classifier(torch.flatten(self.features(x), 1))


class VGG16(_VGG):
    CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]


class VGG19(_VGG):
    CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]
