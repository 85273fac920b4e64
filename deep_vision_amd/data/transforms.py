"""Sample transforms of the PT ImageNet pipeline (R/ResNet/pytorch/data_load.py:72-297), operating
on ``{'image': HWC uint8 ndarray, 'annotation': int}`` samples like the reference.

The reference decodes with cv2; PIL is used here (cv2 is not part of this stack): bilinear
resize, RGB order, alpha dropped, grayscale expanded to 3 channels in ToTensor.
Reference quirks kept for trained-model parity: ``Rescale`` truncates the new size with int();
``RandomCrop`` draws ``randint(0, h - new_h)`` (exclusive upper bound); ``ToTensor`` does **not**
divide by 255, so ``Normalize`` with the ImageNet mean/std acts on 0-255 values
(R/ResNet/pytorch/train.py:315-331); ``ColorJitter`` runs before ToTensor through PIL in a
random order (A21).
"""
from __future__ import annotations

import random

import numpy as np
import torch
from PIL import Image, ImageEnhance

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


class Compose:
    def __init__(self, transforms):
        self.transforms = list(transforms)

    def __call__(self, sample):
        for t in self.transforms:
            sample = t(sample)
        return sample


def _resize(image: np.ndarray, new_h: int, new_w: int) -> np.ndarray:
    return np.asarray(Image.fromarray(image).resize((new_w, new_h), Image.BILINEAR))


class Rescale:
    def __init__(self, output_size):
        assert isinstance(output_size, (int, tuple))
        self.output_size = output_size

    def __call__(self, sample):
        image = sample["image"]
        h, w = image.shape[:2]
        if isinstance(self.output_size, int):
            if h > w:
                new_h, new_w = self.output_size * h / w, self.output_size
            else:
                new_h, new_w = self.output_size, self.output_size * w / h
        else:
            new_h, new_w = self.output_size
        return {**sample, "image": _resize(image, int(new_h), int(new_w))}


class RandomHorizontalFlip:
    def __init__(self, p=0.5):
        self.p = p

    def __call__(self, sample):
        if random.random() < self.p:
            return {**sample, "image": np.ascontiguousarray(np.fliplr(sample["image"]))}
        return sample


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


class RandomCrop:
    def __init__(self, output_size):
        self.output_size = _pair(output_size)

    def __call__(self, sample):
        image = sample["image"]
        h, w = image.shape[:2]
        nh, nw = self.output_size
        top = np.random.randint(0, h - nh) if h > nh else 0
        left = np.random.randint(0, w - nw) if w > nw else 0
        return {**sample, "image": image[top:top + nh, left:left + nw]}


class CenterCrop:
    def __init__(self, output_size):
        self.output_size = _pair(output_size)

    def __call__(self, sample):
        image = sample["image"]
        h, w = image.shape[:2]
        nh, nw = self.output_size
        top, left = (h - nh) // 2, (w - nw) // 2
        return {**sample, "image": image[top:top + nh, left:left + nw]}


class ToTensor:
    """HWC ndarray -> CHW float tensor (values kept in 0-255, like the reference)."""

    def __call__(self, sample):
        image = sample["image"]
        if image.ndim == 2:
            image = np.stack((image,) * 3, axis=-1)
        return {**sample, "image": torch.from_numpy(np.ascontiguousarray(image.transpose(2, 0, 1))).float()}


class Normalize:
    def __init__(self, mean, std):
        self.mean = torch.tensor(mean).view(-1, 1, 1)
        self.std = torch.tensor(std).view(-1, 1, 1)

    def __call__(self, sample):
        return {**sample, "image": (sample["image"] - self.mean) / self.std}


class ColorJitter:
    """Brightness / contrast / saturation (/ hue) jitter in random order through PIL."""

    def __init__(self, brightness=0, contrast=0, saturation=0, hue=0):
        self.brightness, self.contrast, self.saturation, self.hue = brightness, contrast, saturation, hue

    @staticmethod
    def _hue(img, f):
        h, s, v = img.convert("HSV").split()
        h = h.point(lambda x: (x + int(f * 255)) % 256)
        return Image.merge("HSV", (h, s, v)).convert("RGB")

    def get_params(self):
        ts = []
        if self.brightness > 0:
            b = random.uniform(max(0, 1 - self.brightness), 1 + self.brightness)
            ts.append(lambda im: ImageEnhance.Brightness(im).enhance(b))
        if self.contrast > 0:
            c = random.uniform(max(0, 1 - self.contrast), 1 + self.contrast)
            ts.append(lambda im: ImageEnhance.Contrast(im).enhance(c))
        if self.saturation > 0:
            s = random.uniform(max(0, 1 - self.saturation), 1 + self.saturation)
            ts.append(lambda im: ImageEnhance.Color(im).enhance(s))
        if self.hue > 0:
            hf = random.uniform(-self.hue, self.hue)
            ts.append(lambda im: self._hue(im, hf))
        random.shuffle(ts)
        return ts

    def __call__(self, sample):
        image = Image.fromarray(sample["image"], mode="RGB")
        for t in self.get_params():
            image = t(image)
        return {**sample, "image": np.asarray(image)}


def _io():
    try:
        from .. import _io as io

        return io if hasattr(io, "resize_crop") else None
    except ImportError:
        return None


class RescaleCrop:
    """``Rescale(size)`` then ``RandomCrop(crop)`` (train) or ``CenterCrop(crop)`` as ONE native pass
    over the crop window only (deep_vision_amd._io resize_crop: cv2 INTER_LINEAR geometry, the
    reference's cv2.resize, instead of PIL's antialiased bilinear). Same size truncation and crop
    draws as the two-step form (the randint exclusive upper bound quirk included)."""

    def __init__(self, size, crop, random_crop=True):
        self.size, self.crop, self.random_crop = size, _pair(crop), random_crop

    def __call__(self, sample):
        image = sample["image"]
        if image.ndim == 2:
            image = np.stack((image,) * 3, axis=-1)
        h, w = image.shape[:2]
        if h > w:
            nh, nw = int(self.size * h / w), self.size
        else:
            nh, nw = self.size, int(self.size * w / h)
        ch, cw = self.crop
        if self.random_crop:
            top = np.random.randint(0, nh - ch) if nh > ch else 0
            left = np.random.randint(0, nw - cw) if nw > cw else 0
        else:
            top, left = (nh - ch) // 2, (nw - cw) // 2
        io = _io()
        if io is None:  # the two-step form
            r = _resize(image, nh, nw)
            return {**sample, "image": np.ascontiguousarray(r[top:top + ch, left:left + cw])}
        return {**sample, "image": io.resize_crop(image, nh, nw, top, left, ch, cw)}  # strided views read in place


class FastColorJitter(ColorJitter):
    """ColorJitter (brightness / contrast / saturation, random order, the same factor draws) with
    PIL's enhancer arithmetic in one native in-place call per image (deep_vision_amd._io
    color_jitter); hue jitter falls back to PIL."""

    def __call__(self, sample):
        io = _io()
        if io is None or self.hue > 0:
            return super().__call__(sample)
        f, order = [1.0, 1.0, 1.0], []
        for k, amt in enumerate((self.brightness, self.contrast, self.saturation)):
            if amt > 0:
                f[k] = random.uniform(max(0, 1 - amt), 1 + amt)
                order.append(k)
        random.shuffle(order)
        order += [k for k in range(3) if k not in order]
        image = sample["image"]
        if not (image.flags.writeable and image.flags.c_contiguous):
            image = np.ascontiguousarray(image).copy()
        io.color_jitter(image, f, order)
        return {**sample, "image": image}


class JitterDraw(ColorJitter):
    """The draws of ``FastColorJitter`` (same factors, same order shuffle, same RNG calls in the
    same place of the pipeline) without touching the pixels: the factors and order go with the
    sample as ``jitter`` = float32 [f_brightness, f_contrast, f_saturation, op0, op1, op2], and the
    GPU applies them to the uint8 batch (data.device_input.jitter_u8, csrc/elementwise.hip
    u8_jitter: the same bytes as the worker-side jitter). Moves ~12 % of a loader worker's
    per-image CPU time to the device."""

    def __call__(self, sample):
        if self.hue > 0:
            raise ValueError("JitterDraw: hue jitter is host-only (FastColorJitter)")
        f, order = [1.0, 1.0, 1.0], []
        for k, amt in enumerate((self.brightness, self.contrast, self.saturation)):
            if amt > 0:
                f[k] = random.uniform(max(0, 1 - amt), 1 + amt)
                order.append(k)
        random.shuffle(order)
        order += [k for k in range(3) if k not in order]
        return {**sample, "jitter": torch.tensor(f + [float(k) for k in order], dtype=torch.float32)}


class ToUint8:
    """Final step of the device-normalised pipeline (data/device_input.py): the HWC uint8 crop
    as a tensor (grayscale expanded to 3 channels) plus the horizontal-flip draw, which the device
    kernel applies together with ToTensor + Normalize. 150 KB per 224x224 image instead of 602."""

    def __init__(self, flip_p=0.0):
        self.flip_p = flip_p

    def __call__(self, sample):
        image = sample["image"]
        if image.ndim == 2:
            image = np.stack((image,) * 3, axis=-1)
        flip = self.flip_p > 0 and random.random() < self.flip_p
        image = np.ascontiguousarray(image)
        if not image.flags.writeable:  # PIL-backed arrays are read-only
            image = image.copy()
        return {**sample, "image": torch.from_numpy(image), "flip": flip}


def imagenet_train_transform(device_normalize=False, device_jitter=False):
    """R/ResNet/pytorch/train.py:315-324. ``device_normalize``: stop at the uint8 crop + flip
    draw; flip, ToTensor and Normalize run on the GPU (data.device_input). ``device_jitter``
    (with it): the ColorJitter draws stay in the worker, the pixels are jittered on the GPU."""
    if device_normalize:  # native resize-crop + jitter (deep_vision_amd._io)
        jit = JitterDraw if device_jitter else FastColorJitter
        return Compose([RescaleCrop(256, 224), jit(brightness=0.2, contrast=0.2, saturation=0.2, hue=0),
                        ToUint8(flip_p=0.5)])
    return Compose([Rescale(256), RandomHorizontalFlip(0.5), RandomCrop(224),
                    ColorJitter(brightness=0.2, contrast=0.2, saturation=0.2, hue=0), ToTensor(),
                    Normalize(IMAGENET_MEAN, IMAGENET_STD)])


def imagenet_val_transform(device_normalize=False):
    """R/ResNet/pytorch/train.py:326-331."""
    if device_normalize:
        return Compose([RescaleCrop(256, 224, random_crop=False), ToUint8()])
    return Compose([Rescale(256), CenterCrop(224), ToTensor(), Normalize(IMAGENET_MEAN, IMAGENET_STD)])
