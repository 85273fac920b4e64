"""TF1-Keras ImageNet TFRecord input pipeline without TensorFlow.

Reference: R/ResNet/tensorflow/train.py:148-214 (``_parse_function`` over the 9-feature schema,
``create_dataset``: list_files -> TFRecordDataset -> map(parse) -> repeat -> shuffle(10000) ->
batch -> prefetch(1) -> one_hot(label, 1000)) and R/ResNet/tensorflow/data_load.py:35-193
(``preprocess_image``: decode_jpeg -> aspect-preserving bilinear resize of the shorter side to 256
-> training: random_crop 224 + random_flip_left_right / eval: central crop -> RGB mean
subtraction 123.68 / 116.78 / 103.94, no division by a std).

Differences, all deliberate:
  * labels: the builder writes 1..1000 (TF-models convention, 0 = background,
    R/Datasets/ILSVRC2012/build_imagenet_tfrecord.py:515) but the reference one-hots them into
    1000 classes; the reader subtracts 1;
  * records are read through the native TFRecord runtime (csrc/host/io.cpp, CRC-checked), one
    reader per DataLoader worker; the DataLoader's shuffle is a full permutation (a superset of
    ``shuffle(10000)``) and epochs replace ``repeat()``;
  * resize = TF1 ``tf.image.resize_images(BILINEAR, align_corners=False)``: the legacy
    (non half-pixel) source mapping ``src = dst * in / out``, reproduced exactly in numpy.
"""
from __future__ import annotations

import glob
import io
import os
from typing import Optional

import numpy as np
import torch
from torch.utils.data import Dataset

from .tfrecord import TFRecordIndex, decode_example, example_values

CHANNEL_MEANS = (123.68, 116.78, 103.94)  # R/ResNet/tensorflow/data_load.py:41-45
RESIZE_MIN = 256
FEATURES = ("image/height", "image/width", "image/colorspace", "image/channels", "image/class/label",
            "image/class/synset", "image/class/text", "image/filename", "image/encoded")


def smallest_size_at_least(height: int, width: int, resize_min: int = RESIZE_MIN):
    """data_load.py _smallest_size_at_least: float32 scale, truncating int32 casts."""
    scale = np.float32(resize_min) / np.float32(min(height, width))
    return int(np.float32(height) * scale), int(np.float32(width) * scale)


def tf1_resize_bilinear(img: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """TF1 resize_bilinear (align_corners=False, half_pixel_centers=False) of an HWC image;
    float32 result like tf.image.resize_images."""
    in_h, in_w = img.shape[:2]
    src = img.astype(np.float32)

    def axis(n_in, n_out):
        scale = np.float32(n_in) / np.float32(n_out)
        pos = np.arange(n_out, dtype=np.float32) * scale
        lo = np.floor(pos).astype(np.int64)
        hi = np.minimum(lo + 1, n_in - 1)
        frac = (pos - lo).astype(np.float32)
        return lo, hi, frac

    y0, y1, fy = axis(in_h, out_h)
    x0, x1, fx = axis(in_w, out_w)
    top = src[y0][:, x0] + (src[y0][:, x1] - src[y0][:, x0]) * fx[None, :, None]
    bot = src[y1][:, x0] + (src[y1][:, x1] - src[y1][:, x0]) * fx[None, :, None]
    return top + (bot - top) * fy[:, None, None]


def central_crop(img: np.ndarray, h: int, w: int) -> np.ndarray:
    top = (img.shape[0] - h) // 2
    left = (img.shape[1] - w) // 2
    return img[top:top + h, left:left + w]


def decode_jpeg_rgb(data: bytes) -> np.ndarray:
    from PIL import Image

    with Image.open(io.BytesIO(data)) as im:
        return np.asarray(im.convert("RGB"))


def preprocess_image(jpeg: bytes, is_training: bool, out_h: int = 224, out_w: int = 224,
                     rng: Optional[np.random.Generator] = None) -> np.ndarray:
    """data_load.py preprocess_image -> float32 HWC (mean-subtracted)."""
    img = decode_jpeg_rgb(jpeg)
    nh, nw = smallest_size_at_least(img.shape[0], img.shape[1])
    img = tf1_resize_bilinear(img, nh, nw)
    if is_training:
        rng = rng or np.random.default_rng()
        top = int(rng.integers(0, nh - out_h + 1))
        left = int(rng.integers(0, nw - out_w + 1))
        img = img[top:top + out_h, left:left + out_w]
        if rng.random() < 0.5:
            img = img[:, ::-1]
    else:
        img = central_crop(img, out_h, out_w)
    return img - np.asarray(CHANNEL_MEANS, dtype=np.float32)


class ImageNetTFRecordDataset(Dataset):
    """``pattern`` e.g. ``../dataset/tfrecord/tfrecord_train/*`` (reference run_epochs).
    Items: ``{'image': float32 (3, 224, 224), 'annotation': int label in 0..999}``; with
    ``one_hot`` the label is the 1000-vector the reference feeds to categorical_crossentropy."""

    def __init__(self, pattern: str, is_training: bool, one_hot: bool = False, label_offset: int = 1,
                 output_size: int = 224, seed: int = 0):
        files = sorted(glob.glob(pattern)) if not os.path.isdir(pattern) else \
            sorted(os.path.join(pattern, f) for f in os.listdir(pattern))
        if not files:
            raise FileNotFoundError(f"no TFRecord files match {pattern}")
        self.index = TFRecordIndex(files)
        self.is_training = is_training
        self.one_hot = one_hot
        self.label_offset = label_offset
        self.size = output_size
        self.seed = seed
        self._rng = None

    def __len__(self):
        return len(self.index)

    def parse(self, i: int) -> dict:
        """The 9 features of ``_parse_function`` (missing optional ones come back as None)."""
        ex = decode_example(self.index[i])
        out = {}
        for k in FEATURES:
            v = example_values(ex, k)
            out[k] = None if not v else v[0]
        return out

    def __getitem__(self, i: int):
        if self._rng is None:  # per worker process
            info = torch.utils.data.get_worker_info()
            self._rng = np.random.default_rng(self.seed + (info.id if info is not None else 0) + 7919 * os.getpid())
        f = self.parse(i)
        if f["image/encoded"] is None or f["image/class/label"] is None:
            raise ValueError(f"record {i} lacks image/encoded or image/class/label")
        img = preprocess_image(f["image/encoded"], self.is_training, self.size, self.size, self._rng)
        label = int(f["image/class/label"]) - self.label_offset
        t = torch.from_numpy(np.ascontiguousarray(img.transpose(2, 0, 1)))
        if self.one_hot:
            lab = torch.zeros(1000)
            lab[label] = 1.0
            return {"image": t, "annotation": lab}
        return {"image": t, "annotation": label}
