"""DCGAN (R/DCGAN/tensorflow/models.py:8-65) and CycleGAN (R/CycleGAN/tensorflow/models.py:8-104).

Keras semantics kept: 'same' padding (asymmetric at stride 2 / even kernels), Conv2DTranspose
'same' output geometry (input x stride, top/left pad (k - s) // 2), BatchNormalization
eps 1e-3 / momentum .99 (torch .01), LeakyReLU default alpha 0.3 (DCGAN), NHWC flatten order
before Dense layers (free in the native NHWC layout). Parameter counts: DCGAN G 2,305,472 /
D 212,865; CycleGAN G 11,383,427 / D 2,765,633 (pinned in tests).

CycleGAN keeps the reference's BatchNorm (not InstanceNorm) and plain ``inputs + x`` residual
blocks; reflection padding is explicit.
"""
from __future__ import annotations

import torch
import torch.nn as tnn

from .. import nn
from .. import ops as F


def _bn(c):
    return nn.BatchNorm2d(c, eps=1e-3, momentum=0.01)


def _flatten_nhwc(x):
    """Keras Flatten of an NHWC feature map: (h, w, c) order (a free view of the native layout)."""
    return x.permute(0, 2, 3, 1).reshape(x.shape[0], -1)


# ----------------------------------------- DCGAN -----------------------------------------
class DCGANGenerator(tnn.Module):
    """Dense(100 -> 7*7*256, no bias) -> BN -> LeakyReLU(.3) -> reshape (7, 7, 256) ->
    ConvT 5x5/1 128 -> BN -> LReLU -> ConvT 5x5/2 64 -> BN -> LReLU -> ConvT 5x5/2 1 -> tanh."""

    def __init__(self, noise_dim=100):
        super().__init__()
        self.noise_dim = noise_dim
        self.dense = nn.Linear(noise_dim, 7 * 7 * 256, bias=False)
        self.bn0 = nn.BatchNorm2d(7 * 7 * 256, eps=1e-3, momentum=0.01)  # Keras BN over the dense features
        self.deconv1 = nn.ConvTranspose2d(256, 128, 5, stride=1, padding="same_keras", bias=False)
        self.bn1 = _bn(128)
        self.deconv2 = nn.ConvTranspose2d(128, 64, 5, stride=2, padding="same_keras", bias=False)
        self.bn2 = _bn(64)
        self.deconv3 = nn.ConvTranspose2d(64, 1, 5, stride=2, padding="same_keras", bias=False)

    def forward(self, z):
        x = self.dense(z)
        N = x.shape[0]
        x = F.batch_norm_act(x.reshape(N, -1, 1, 1), self.bn0, "leaky", 0.3)
        # Keras Reshape((7, 7, 256)) of the feature vector = an NHWC tensor
        x = x.reshape(N, 7, 7, 256).permute(0, 3, 1, 2)
        x = F.batch_norm_act(self.deconv1(x), self.bn1, "leaky", 0.3)
        x = F.batch_norm_act(self.deconv2(x), self.bn2, "leaky", 0.3)
        return F.activation(self.deconv3(x), "tanh")


class DCGANDiscriminator(tnn.Module):
    """Conv 5x5/2 64 -> LReLU(.3) -> Dropout .3 -> Conv 5x5/2 128 -> LReLU -> Dropout -> Dense 1."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 64, 5, stride=2, padding="same_keras")
        self.conv2 = nn.Conv2d(64, 128, 5, stride=2, padding="same_keras")
        self.drop = nn.Dropout(0.3)
        self.dense = nn.Linear(7 * 7 * 128, 1)

    def _conv_act(self, conv, x):
        return F.conv2d(x, conv.weight, conv.bias, conv.stride, conv.native_padding(x.shape[2], x.shape[3]),
                        act="leaky", slope=0.3)

    def forward(self, x):
        x = self.drop(self._conv_act(self.conv1, x))
        x = self.drop(self._conv_act(self.conv2, x))
        return self.dense(_flatten_nhwc(x))


# ---------------------------------------- CycleGAN ----------------------------------------
def _rpad(pad_module):
    """(top, left) of a symmetric nn.ReflectionPad2d (padding = (left, right, top, bottom))."""
    l, r, t, b = pad_module.padding
    assert l == r and t == b, "asymmetric reflection padding"
    return (t, l)

class ResNetBlock(tnn.Module):
    """reflect-pad 1 -> conv3x3 -> BN -> ReLU -> reflect-pad 1 -> conv3x3 -> BN, + input (models.py:17-38)."""

    def __init__(self, dim):
        super().__init__()
        self.pad = nn.ReflectionPad2d(1)
        self.conv1 = nn.Conv2d(dim, dim, 3, bias=False)
        self.bn1 = _bn(dim)
        self.conv2 = nn.Conv2d(dim, dim, 3, bias=False)
        self.bn2 = _bn(dim)

    def forward(self, x):
        # ReflectionPad2d(1) is fused into each conv's im2col gather (mirrored taps, no padded copy)
        p = _rpad(self.pad)
        y = F.conv_bn_act(x, self.conv1, self.bn1, "relu", reflect_pad=p)
        return F.conv_bn_act(y, self.conv2, self.bn2, None, residual=x, reflect_pad=p)


class CycleGANGenerator(tnn.Module):
    def __init__(self, n_blocks=9, channels=3):
        super().__init__()
        self.pad_in = nn.ReflectionPad2d(3)
        self.conv_in = nn.Conv2d(channels, 64, 7, bias=False)
        self.bn_in = _bn(64)
        self.down1 = nn.Conv2d(64, 128, 3, stride=2, padding="same_keras", bias=False)
        self.bn_d1 = _bn(128)
        self.down2 = nn.Conv2d(128, 256, 3, stride=2, padding="same_keras", bias=False)
        self.bn_d2 = _bn(256)
        self.blocks = tnn.Sequential(*[ResNetBlock(256) for _ in range(n_blocks)])
        self.up1 = nn.ConvTranspose2d(256, 128, 3, stride=2, padding="same_keras", bias=False)
        self.bn_u1 = _bn(128)
        self.up2 = nn.ConvTranspose2d(128, 64, 3, stride=2, padding="same_keras", bias=False)
        self.bn_u2 = _bn(64)
        self.pad_out = nn.ReflectionPad2d(3)
        self.conv_out = nn.Conv2d(64, channels, 7)

    def forward(self, x):
        x = F.conv_bn_act(x, self.conv_in, self.bn_in, "relu", reflect_pad=_rpad(self.pad_in))
        x = F.conv_bn_act(x, self.down1, self.bn_d1, "relu")
        x = F.conv_bn_act(x, self.down2, self.bn_d2, "relu")
        x = self.blocks(x)
        x = F.batch_norm_act(self.up1(x), self.bn_u1, "relu")
        x = F.batch_norm_act(self.up2(x), self.bn_u2, "relu")
        x = F.conv2d(x, self.conv_out.weight, self.conv_out.bias, 1, _rpad(self.pad_out), pad_mode="reflect")
        return F.activation(x, "tanh")


class CycleGANDiscriminator(tnn.Module):
    """70x70 PatchGAN: conv4x4/2 64 -> LReLU(.2) -> [conv4x4 -> BN -> LReLU(.2)] x3 (128/2, 256/2,
    512/1) -> conv4x4/1 1 (models.py:81-104)."""

    def __init__(self, channels=3):
        super().__init__()
        self.conv1 = nn.Conv2d(channels, 64, 4, stride=2, padding="same_keras")
        self.conv2 = nn.Conv2d(64, 128, 4, stride=2, padding="same_keras", bias=False)
        self.bn2 = _bn(128)
        self.conv3 = nn.Conv2d(128, 256, 4, stride=2, padding="same_keras", bias=False)
        self.bn3 = _bn(256)
        self.conv4 = nn.Conv2d(256, 512, 4, stride=1, padding="same_keras", bias=False)
        self.bn4 = _bn(512)
        self.conv5 = nn.Conv2d(512, 1, 4, stride=1, padding="same_keras")

    def forward(self, x):
        c = self.conv1
        x = F.conv2d(x, c.weight, c.bias, c.stride, c.native_padding(x.shape[2], x.shape[3]), act="leaky", slope=0.2)
        x = F.conv_bn_act(x, self.conv2, self.bn2, "leaky", 0.2)
        x = F.conv_bn_act(x, self.conv3, self.bn3, "leaky", 0.2)
        x = F.conv_bn_act(x, self.conv4, self.bn4, "leaky", 0.2)
        return self.conv5(x)


def dcgan(**kw):
    return torch.nn.ModuleDict({"generator": DCGANGenerator(**kw), "discriminator": DCGANDiscriminator()})


def cyclegan(n_blocks=9):
    """Two generators (G: A->B, F: B->A) and two discriminators (D_A, D_B), R/CycleGAN/tensorflow/train.py:122-131."""
    return torch.nn.ModuleDict({"generator_g": CycleGANGenerator(n_blocks), "generator_f": CycleGANGenerator(n_blocks),
                                "discriminator_x": CycleGANDiscriminator(), "discriminator_y": CycleGANDiscriminator()})
