"""Device-side end of the image input pipeline.

The reference's workers decode, resize, flip, crop, jitter, convert to float CHW and normalise on
the CPU (R/ResNet/pytorch/data_load.py:72-297, R/ResNet/pytorch/train.py:315-331) and the batch
crosses PCIe as fp32: 602 KB per 224x224 image, ~7.7 GB/s per GPU at 12.9k img/s. Here the workers
stop at the uint8 HWC crop (``transforms.ToUint8``: 150 KB, a quarter of the bytes) plus a flip
flag; the trainer copies that batch to the GPU and one kernel (csrc/elementwise.hip
``u8_normalize``) mirrors flipped samples, normalises and writes the bf16 NCHW network input.

Normalisation constants: ``(scale, mean, std)`` with the reference quirk by default -- its
ToTensor keeps 0-255 values and Normalize subtracts the ImageNet mean / divides by the std on
that range (scale 1). The flip is applied to the crop instead of the resized image before the
crop; since the crop offset is uniform that is the same distribution (up to the reference's
exclusive randint upper bound).
"""
from __future__ import annotations

import torch

from ..ops.common import BF16, lib, native, ptr, stream_handle
from .transforms import IMAGENET_MEAN, IMAGENET_STD

REFERENCE_NORM = (1.0, IMAGENET_MEAN, IMAGENET_STD)  # ToTensor without /255 (reference quirk)


def jitter_u8(img, jitter):
    """ColorJitter of ``transforms.JitterDraw`` applied IN PLACE to a uint8 [N, H, W, 3] batch:
    ``jitter`` float32 [N, 6] (factors, order). GPU: one native launch (csrc/elementwise.hip
    u8_jitter); CPU: the worker-side native jitter (deep_vision_amd._io), per image. Both give the
    bytes ``FastColorJitter`` gives."""
    N, H, W, C = img.shape
    if C != 3 or not img.is_contiguous():
        raise ValueError("jitter_u8: a contiguous [N, H, W, 3] uint8 batch")
    if native(img):
        prm = jitter.to(device=img.device, dtype=torch.float32).contiguous()
        lib().u8_jitter(ptr(img), ptr(prm), N, H * W, stream_handle())
        return img
    from .. import _io

    host = img if img.device.type == "cpu" else img.cpu()
    j = jitter.cpu()
    for n in range(N):
        _io.color_jitter(host[n].numpy(), [float(v) for v in j[n, :3]], [int(v) for v in j[n, 3:]])
    if host is not img:
        img.copy_(host)
    return img


def normalize_u8(img, flip=None, norm=REFERENCE_NORM, out_dtype=None, jitter=None):
    """``img`` uint8 [N, H, W, C] (on any device), ``flip`` bool/uint8 [N] or None ->
    normalised NCHW: bf16 from the native kernel on the GPU, fp32 (or ``out_dtype``) on the CPU.
    ``jitter`` ([N, 6], ``transforms.JitterDraw``): ColorJitter first, in place on ``img``."""
    scale, mean, std = norm
    N, H, W, C = img.shape
    if jitter is not None:
        img = jitter_u8(img.contiguous(), jitter)
    if native(img):
        x = img.contiguous()
        f = flip.to(device=img.device, dtype=torch.uint8).contiguous() if flip is not None else None
        y = torch.empty((N, C, H, W), dtype=BF16, device=img.device)
        lib().u8_normalize(ptr(x), ptr(f), ptr(y), N, C, H, W, float(scale), [float(v) for v in mean[:C]],
                           [float(v) for v in std[:C]], stream_handle())
        return y if out_dtype in (None, BF16) else y.to(out_dtype)
    x = img.permute(0, 3, 1, 2).float() * scale
    if flip is not None:
        fl = flip.to(torch.bool).view(N, 1, 1, 1)
        x = torch.where(fl, x.flip(3), x)
    m = torch.tensor(mean[:C], dtype=torch.float32).view(1, C, 1, 1)
    s = torch.tensor(std[:C], dtype=torch.float32).view(1, C, 1, 1)
    y = (x - m) / s
    return y if out_dtype is None else y.to(out_dtype)


def batch_images(data, device, non_blocking=True):
    """The network input of a loader batch: float tensors are moved as they are; uint8 HWC crops
    (``ToUint8``) are moved as bytes and normalised on the device."""
    img = data["image"]
    if img.dtype == torch.uint8 and img.dim() == 4:
        img = img.to(device, non_blocking=non_blocking)
        flip, jit = data.get("flip"), data.get("jitter")
        if flip is not None:
            flip = flip.to(device, non_blocking=non_blocking)
        return normalize_u8(img, flip, jitter=jit)
    return img.to(device, non_blocking=non_blocking)
