"""CenterNet ("Objects as Points") targets and decoding.

The reference preprocessing is unfinished (``generate_2d_guassian`` returns zeros
early, ``make_label`` references an undefined attribute, R/ObjectsAsPoints/tensorflow/
preprocess.py:138,201-221), so the targets follow the paper (Zhou et al. 2019, sec. 3):
per class a Gaussian splat at each object centre on the stride-4 grid with the CornerNet
size-adaptive radius, plus size (w, h in output pixels) and sub-pixel offset regression
targets at the centre cell with a mask. Dense (C, g, g) / (2, g, g) maps, so the losses run
through the fused pointwise kernels (focal + masked L1).
"""
from __future__ import annotations

import numpy as np


def gaussian_radius(h, w, min_overlap=0.7):
    """CornerNet radius such that a box shifted by r keeps IoU >= min_overlap."""
    a1, b1 = 1, h + w
    c1 = w * h * (1 - min_overlap) / (1 + min_overlap)
    r1 = (b1 + np.sqrt(b1 ** 2 - 4 * a1 * c1)) / 2
    a2, b2 = 4, 2 * (h + w)
    c2 = (1 - min_overlap) * w * h
    r2 = (b2 + np.sqrt(b2 ** 2 - 4 * a2 * c2)) / 2
    a3, b3 = 4 * min_overlap, -2 * min_overlap * (h + w)
    c3 = (min_overlap - 1) * w * h
    r3 = (b3 + np.sqrt(b3 ** 2 - 4 * a3 * c3)) / 2
    return min(r1, r2, r3)


def draw_gaussian(hm, cx, cy, radius):
    d = 2 * radius + 1
    sigma = d / 6
    yy, xx = np.ogrid[-radius:radius + 1, -radius:radius + 1]
    g = np.exp(-(xx * xx + yy * yy) / (2 * sigma * sigma))
    H, W = hm.shape
    l, r = min(cx, radius), min(W - cx, radius + 1)
    t, b = min(cy, radius), min(H - cy, radius + 1)
    region = hm[cy - t:cy + b, cx - l:cx + r]
    np.maximum(region, g[radius - t:radius + b, radius - l:radius + r], out=region)
    return hm


def encode(boxes, classes, num_classes, out_size=64):
    """boxes (K, 4) normalised x1y1x2y2 -> heatmap (C, g, g), size (2, g, g), offset (2, g, g),
    mask (2, g, g) (1 at object centres, duplicated over the two regression channels)."""
    g = out_size
    hm = np.zeros((num_classes, g, g), np.float32)
    wh = np.zeros((2, g, g), np.float32)
    off = np.zeros((2, g, g), np.float32)
    mask = np.zeros((2, g, g), np.float32)
    for (x1, y1, x2, y2), c in zip(np.asarray(boxes, np.float32).reshape(-1, 4), classes):
        w, h = (x2 - x1) * g, (y2 - y1) * g
        if w <= 0 or h <= 0:
            continue
        cx, cy = (x1 + x2) / 2 * g, (y1 + y2) / 2 * g
        ix, iy = min(int(cx), g - 1), min(int(cy), g - 1)
        r = max(0, int(gaussian_radius(np.ceil(h), np.ceil(w))))
        draw_gaussian(hm[int(c)], ix, iy, r)
        wh[:, iy, ix] = (w, h)
        off[:, iy, ix] = (cx - ix, cy - iy)
        mask[:, iy, ix] = 1.0
    return hm, wh, off, mask


class SyntheticCenterNetDataset:
    def __init__(self, n=64, num_classes=80, size=256, seed=0):
        self.n, self.num_classes, self.size, self.seed = n, num_classes, size, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        from .yolo import synthetic_sample

        rng = np.random.default_rng((self.seed, i))
        img, boxes, classes = synthetic_sample(rng, self.num_classes, self.size)
        return img, encode(boxes, classes, self.num_classes, self.size // 4)


def collate(batch):
    import torch

    imgs = torch.from_numpy(np.stack([b[0] for b in batch]))
    tg = tuple(torch.from_numpy(np.stack([b[1][k] for b in batch])) for k in range(4))
    return imgs, tg


def decode(heatmap_logits, size, offset, k=100):
    """Top-k peaks (3x3 max-pool NMS) -> (N, k, 6): x1, y1, x2, y2 (output pixels), score, class."""
    import torch
    import torch.nn.functional as TF

    hm = torch.sigmoid(heatmap_logits.float())
    keep = (TF.max_pool2d(hm, 3, 1, 1) == hm).float()
    hm = hm * keep
    N, C, H, W = hm.shape
    scores, idx = hm.view(N, -1).topk(k)
    cls = idx // (H * W)
    pix = idx % (H * W)
    ys, xs = (pix // W).float(), (pix % W).float()
    g = lambda t: t.float().view(N, 2, -1).gather(2, pix.unsqueeze(1).expand(N, 2, k))  # noqa: E731
    wh, of = g(size), g(offset)
    cx, cy = xs + of[:, 0], ys + of[:, 1]
    return torch.stack([cx - wh[:, 0] / 2, cy - wh[:, 1] / 2, cx + wh[:, 0] / 2, cy + wh[:, 1] / 2, scores,
                        cls.float()], -1)
