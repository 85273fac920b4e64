"""Classification datasets: MNIST IDX (R/LeNet/pytorch/data_load.py:12-57), flattened ImageNet-2012
(R/ResNet/pytorch/data_load.py:20-69) and synthetic on-device data of the same shapes.

Samples are dicts like the reference's: MNIST ``{'image', 'label'}``, ImageNet
``{'image', 'annotation'}``. The reference repository ships the MNIST *labels* only (images
are stripped, R/.MISSING_LARGE_BLOBS:3-4); ``MnistDataset(..., synthetic_images=True)`` pairs
the real label files with synthetic digits so the LeNet plumbing still runs end to end.
"""
from __future__ import annotations

import os
from os.path import isfile, join

import numpy as np
import torch
from PIL import Image
from torch.utils.data import Dataset

MNIST_MEAN, MNIST_STD = 0.1307, 0.3081


def read_idx(path: str) -> np.ndarray:
    """IDX file (big-endian magic: 0x0000 08 <ndim>) -> uint8 ndarray."""
    with open(path, "rb") as f:
        b = f.read()
    magic = int.from_bytes(b[0:4], "big")
    if magic >> 8 != 0x08:
        raise ValueError(f"{path}: not an unsigned-byte IDX file (magic {magic:#x})")
    ndim = magic & 0xFF
    dims = [int.from_bytes(b[4 + 4 * i: 8 + 4 * i], "big") for i in range(ndim)]
    off = 4 + 4 * ndim
    return np.frombuffer(b, dtype=np.uint8, count=int(np.prod(dims)), offset=off).reshape(dims)


def write_idx(path: str, arr: np.ndarray) -> None:
    arr = np.ascontiguousarray(arr, dtype=np.uint8)
    with open(path, "wb") as f:
        f.write((0x0800 | arr.ndim).to_bytes(4, "big"))
        for d in arr.shape:
            f.write(int(d).to_bytes(4, "big"))
        f.write(arr.tobytes())


def synthetic_digits(labels: np.ndarray, seed: int = 0) -> np.ndarray:
    """28x28 uint8 images whose content depends on the label (a learnable synthetic MNIST)."""
    rng = np.random.default_rng(seed)
    n = len(labels)
    protos = rng.integers(0, 256, (10, 28, 28)).astype(np.float32)
    noise = rng.normal(0, 40, (n, 28, 28)).astype(np.float32)
    return np.clip(protos[labels] + noise, 0, 255).astype(np.uint8)


class MnistDataset(Dataset):
    """Pads 28 -> 32 and normalises with the MNIST mean/std on raw 0-255 values (like the
    reference); everything is kept in memory as one tensor."""

    def __init__(self, images_path, labels_path, mean=(MNIST_MEAN,), std=(MNIST_STD,), synthetic_images=False,
                 pad=2, scale=1.0):
        labels = read_idx(labels_path) if labels_path and os.path.exists(labels_path) else None
        if images_path and os.path.exists(images_path):
            images = read_idx(images_path)
            if labels is None:
                raise FileNotFoundError(labels_path)
        elif synthetic_images:
            if labels is None:
                labels = np.random.default_rng(0).integers(0, 10, 1000).astype(np.uint8)
            images = synthetic_digits(labels.astype(np.int64))
        else:
            raise FileNotFoundError(images_path)
        x = torch.from_numpy(images.astype(np.float32) / scale)
        if pad:
            x = torch.nn.functional.pad(x, (pad, pad, pad, pad))
        x = x.unsqueeze(1)
        self.images = (x - mean[0]) / std[0]
        self.labels = torch.from_numpy(labels.astype(np.int64))

    def __len__(self):
        return len(self.labels)

    def __getitem__(self, idx):
        return {"image": self.images[idx], "label": self.labels[idx]}


def read_synsets(labels_file: str | None = None):
    """``synsets.txt`` lines ``nXXXXXXXX name ...`` -> (label->idx, idx->name). ``None`` reads the
    packaged copy (data.imagenet_meta). Names keep the reference's space-dropping
    join (R/ResNet/pytorch/data_load.py:27-44)."""
    if labels_file is None:
        from .imagenet_meta import render

        lines = render("synsets.txt").split("\n")
    else:
        with open(labels_file) as f:
            lines = f.read().split("\n")
    label_to_idx, idx_to_name = {}, {}
    for idx, line in enumerate(l for l in lines if l.strip()):
        parts = line.strip().split(" ")
        label_to_idx[parts[0]] = idx
        idx_to_name[idx] = "".join(parts[1:])
    return label_to_idx, idx_to_name


def _arrow_rgb_view(im):
    """The decoded RGB image's own buffer as an (H, W, 3) view with pixel stride 4 (Pillow keeps
    RGB as RGBX; the Arrow C data export hands that memory over without the ``tobytes`` copy that
    ``np.asarray(im)`` makes, and holds a reference to it). None when unavailable."""
    try:
        import pyarrow as pa

        a = pa.array(im)
        v = a.flatten().to_numpy(zero_copy_only=True)
    except Exception:  # no pyarrow, an older Pillow, a multi-block image
        return None
    w, h = im.size
    if v.size != w * h * 4:
        return None
    return v.reshape(h, w, 4)[:, :, :3]


def load_rgb(path: str, min_side: int | None = None, zero_copy: bool = False) -> np.ndarray:
    """Decode to HWC uint8 RGB (alpha dropped; grayscale stays 2-D for ToTensor to expand).
    ``min_side``: a JPEG is decoded at the smallest DCT scale (1/2, 1/4, 1/8) whose shorter side is
    still >= min_side (PIL draft): the pipeline rescales to that side next anyway, and large images
    decode several times faster. ``zero_copy``: an RGB image comes back as a read-only strided view
    of the decoder's buffer (the native resize-crop reads it in place; others copy as needed)."""
    with Image.open(path) as im:
        if min_side and im.format == "JPEG":
            w, h = im.size
            s = min(w, h)
            if s >= 2 * min_side:
                im.draft("RGB", (-(-w * min_side // s), -(-h * min_side // s)))
        if im.mode in ("RGBA", "P", "CMYK", "LA"):
            im = im.convert("RGB")
        if zero_copy and im.mode == "RGB":
            im.load()
            arr = _arrow_rgb_view(im)
            if arr is not None:
                return arr
        arr = np.asarray(im)
    if arr.ndim == 3 and arr.shape[2] == 4:
        arr = arr[:, :, :3]
    return arr


class ImageNet2012Dataset(Dataset):
    """A flattened directory (``nXXXXXXXX_<file>.JPEG``, T1c) with labels from the synset prefix."""

    def __init__(self, root_dir, labels_file=None, transform=None, decode_min_side=None, zero_copy=None):
        self.root_dir = root_dir
        self.decode_min_side = decode_min_side  # load_rgb min_side: reduced-scale JPEG decode
        # load_rgb zero_copy (opt-in): measured no faster per worker and 5-15 % slower with 4-16 loader
        # workers than the copying decode (profiles/input_pipeline_box.json: pyarrow per worker process)
        self.zero_copy = bool(zero_copy)
        self.images = sorted(f for f in os.listdir(root_dir) if isfile(join(root_dir, f)))
        self.transform = transform
        self.label_to_idx, self.idx_to_name = read_synsets(labels_file)

    def __len__(self):
        return len(self.images)

    def __getitem__(self, idx):
        name = self.images[idx]
        sample = {"image": load_rgb(join(self.root_dir, name), self.decode_min_side, zero_copy=self.zero_copy),
                  "annotation": self.label_to_idx[name.split("_")[0]]}
        return self.transform(sample) if self.transform else sample


class SyntheticClassification(Dataset):
    """Deterministic random images (float CHW) and labels; ``key`` names the label field."""

    def __init__(self, n=1024, shape=(3, 224, 224), num_classes=1000, key="annotation", seed=0):
        self.n, self.shape, self.num_classes, self.key, self.seed = n, tuple(shape), num_classes, key, seed

    def __len__(self):
        return self.n

    def __getitem__(self, idx):
        g = torch.Generator().manual_seed(self.seed * 1000003 + idx)
        label = int(torch.randint(0, self.num_classes, (1,), generator=g))
        # class-dependent mean so a model can fit it (smoke training / convergence tests)
        img = torch.randn(self.shape, generator=g) + (label % 7 - 3) * 0.5
        return {"image": img, self.key: label}


class DeviceSyntheticBatches:
    """On-device synthetic batches (no host pipeline in the timed region; bench / --synthetic)."""

    def __init__(self, batch, shape, num_classes, steps, device, dtype=torch.float32, seed=0):
        g = torch.Generator(device="cpu").manual_seed(seed)
        self.x = torch.randn((batch, *shape), generator=g).to(device=device, dtype=dtype)
        self.y = torch.randint(0, num_classes, (batch,), generator=g).to(device)
        self.steps = steps

    def __len__(self):
        return self.steps

    def __iter__(self):
        for _ in range(self.steps):
            yield {"image": self.x, "annotation": self.y, "label": self.y}
