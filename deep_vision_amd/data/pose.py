"""Stacked-Hourglass input pipeline (R/Hourglass/tensorflow/preprocess.py:4-190).

ROI crop around the visible keypoints with a margin of ``margin x body height`` (random
0.1-0.3 when training, 0.2 otherwise), resize to 256, scale to [-1, 1], and 16 Gaussian
heatmaps of 64x64 (sigma 1, 7x7 patch, **peak 12**, visibility 0 -> empty map). The heatmap
rendering is vectorised numpy (the reference scatters point by point in a tf.function).

The MPII TFRecord schema expected here is the *reader's* one (parts x/y/v as int64 lists,
center x/y int64, scale float) -- the reference writer emits float parts through an Int64List
and no center/scale; data/builders.py writes this schema.
"""
from __future__ import annotations

import numpy as np

from .yolo import decode_image, resize


def gaussian_heatmap(height, width, y0, x0, visibility=2, sigma=1, scale=12.0):
    hm = np.zeros((height, width), np.float32)
    xmin, ymin, xmax, ymax = x0 - 3 * sigma, y0 - 3 * sigma, x0 + 3 * sigma, y0 + 3 * sigma
    if xmin >= width or ymin >= height or xmax < 0 or ymax < 0 or visibility == 0:
        return hm
    size = 6 * sigma + 1
    yy, xx = np.mgrid[0:size, 0:size]
    c = size // 2
    patch = (np.exp(-((xx - c) ** 2 + (yy - c) ** 2) / (sigma ** 2 * 2)) * scale).astype(np.float32)
    # the reference's patch bounds exclude the xmax/ymax column (range(patch_min, patch_max))
    pxmin, pymin = max(0, -xmin), max(0, -ymin)
    pxmax, pymax = min(xmax, width) - xmin, min(ymax, height) - ymin
    hxmin, hymin = max(0, xmin), max(0, ymin)
    hm[hymin:hymin + (pymax - pymin), hxmin:hxmin + (pxmax - pxmin)] = patch[pymin:pymax, pxmin:pxmax]
    return hm


def make_heatmaps(kx, ky, v, shape=(64, 64, 16)):
    """(64, 64, 16) HWC like the reference (transposed to CHW by the dataset)."""
    x = np.round(np.asarray(kx) * shape[0]).astype(np.int64)
    y = np.round(np.asarray(ky) * shape[1]).astype(np.int64)
    maps = [gaussian_heatmap(shape[1], shape[0], int(y[i]), int(x[i]), int(v[i])) for i in range(shape[2])]
    return np.stack(maps, -1)


def crop_roi(image, kx, ky, scale, margin=0.2):
    h, w = image.shape[:2]
    kx = np.asarray(kx, np.int64)
    ky = np.asarray(ky, np.int64)
    body = scale * 200.0
    mx, my = kx[kx != -1], ky[ky != -1]
    xmin = mx.min() - int(body * margin)
    xmax = mx.max() + int(body * margin)
    ymin = my.min() - int(body * margin)
    ymax = my.max() + int(body * margin)
    exmin, eymin = max(xmin, 0), max(ymin, 0)
    exmax, eymax = min(xmax, w), min(ymax, h)
    crop = image[eymin:eymax, exmin:exmax]
    nh, nw = crop.shape[:2]
    return crop, (kx - exmin) / nw, (ky - eymin) / nh


class MPIITFRecordDataset:
    def __init__(self, files, is_train, image_shape=(256, 256), heatmap_shape=(64, 64, 16), encode_on_device=False):
        from .tfrecord import TFRecordIndex

        self.encode_on_device = encode_on_device  # ship keypoint cells; ops.labels.render_heatmaps on the GPU
        self.index = TFRecordIndex(files)
        self.is_train = is_train
        self.image_shape = tuple(image_shape)
        self.heatmap_shape = tuple(heatmap_shape)

    def __len__(self):
        return len(self.index)

    def __getitem__(self, i):
        from .tfrecord import decode_example, example_values

        ex = decode_example(self.index[i])
        image = decode_image(example_values(ex, "image/encoded")[0])
        kx = example_values(ex, "image/object/parts/x")
        ky = example_values(ex, "image/object/parts/y")
        v = example_values(ex, "image/object/parts/v")
        scale = example_values(ex, "image/object/scale")[0]
        margin = float(np.random.uniform(0.1, 0.3)) if self.is_train else 0.2
        image, kx, ky = crop_roi(image, kx, ky, scale, margin)
        image = resize(image, self.image_shape).astype(np.float32) / 127.5 - 1
        if self.encode_on_device:
            return np.ascontiguousarray(image.transpose(2, 0, 1)), _raw_keypoints(kx, ky, v, self.heatmap_shape)
        hm = make_heatmaps(kx, ky, v, self.heatmap_shape)
        return np.ascontiguousarray(image.transpose(2, 0, 1)), np.ascontiguousarray(hm.transpose(2, 0, 1))


def _raw_keypoints(kx, ky, v, shape):
    from ..ops.labels import keypoint_cells

    px, py = keypoint_cells(kx, ky, shape)
    return px, py, np.asarray(v, np.int32)


def collate_raw(batch):
    """Collate of an ``encode_on_device`` dataset: images + {'kind': 'pose', px, py, vis (N, J)}."""
    import torch

    imgs = torch.from_numpy(np.stack([b[0] for b in batch]))
    px, py, vis = (torch.from_numpy(np.stack([b[1][k] for b in batch])) for k in range(3))
    return imgs, {"kind": "pose", "px": px, "py": py, "vis": vis}


class SyntheticPoseDataset:
    def __init__(self, n=64, image_size=256, heatmap_shape=(64, 64, 16), seed=0, encode_on_device=False):
        self.n, self.image_size, self.heatmap_shape, self.seed = n, image_size, heatmap_shape, seed
        self.encode_on_device = encode_on_device

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        rng = np.random.default_rng((self.seed, i))
        img = rng.uniform(-1, 1, (3, self.image_size, self.image_size)).astype(np.float32)
        k = self.heatmap_shape[2]
        kx, ky, v = rng.uniform(0.1, 0.9, k), rng.uniform(0.1, 0.9, k), rng.integers(0, 3, k)
        if self.encode_on_device:
            return img, _raw_keypoints(kx, ky, v, self.heatmap_shape)
        hm = make_heatmaps(kx, ky, v, self.heatmap_shape)
        return img, np.ascontiguousarray(hm.transpose(2, 0, 1))


def keypoints_from_heatmaps(heatmaps):
    """Argmax per heatmap with a quarter-pixel shift toward the larger neighbour
    (R/Hourglass/tensorflow/demo_hourglass_pose.ipynb cells 2-8). heatmaps (K, H, W) ->
    (K, 3) = (x, y, peak) in heatmap pixels."""
    hm = np.asarray(heatmaps, np.float32)
    K, H, W = hm.shape
    out = np.zeros((K, 3), np.float32)
    for k in range(K):
        idx = int(np.argmax(hm[k]))
        y, x = divmod(idx, W)
        fx, fy = float(x), float(y)
        if 0 < x < W - 1:
            fx += 0.25 * np.sign(hm[k, y, x + 1] - hm[k, y, x - 1])
        if 0 < y < H - 1:
            fy += 0.25 * np.sign(hm[k, y + 1, x] - hm[k, y - 1, x])
        out[k] = (fx, fy, hm[k, y, x])
    return out
