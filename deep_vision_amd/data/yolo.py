"""YOLOv3 label encoding and box augmentation (R/YOLO/tensorflow/preprocess.py:20-175).

``encode_labels`` turns one image's ground truth -- normalised (xmin, ymin, xmax, ymax) boxes and
integer classes -- into the three per-scale training targets (g, g, 3, 5+C) =
(cx, cy, w, h, objectness, one-hot class), assigning each box to its best anchor by
width/height IoU (find_best_anchor) and to the grid cell containing its centre. Vectorised
numpy (the reference loops in a tf.function); duplicate cell/anchor assignments keep the last
box, as tensor_scatter_nd_update does on this path.
"""
from __future__ import annotations

import numpy as np

from ..models.yolov3 import ANCHOR_MASKS, ANCHORS_WH

GRIDS = (52, 26, 13)  # stride 8 / 16 / 32 of a 416 input


def find_best_anchor(boxes, anchors_wh=ANCHORS_WH):
    """(K, 4) x1y1x2y2 -> (K,) index of the anchor with the highest width/height IoU."""
    wh = (boxes[:, 2:4] - boxes[:, 0:2])[:, None, :]
    inter = np.minimum(wh[..., 0], anchors_wh[:, 0]) * np.minimum(wh[..., 1], anchors_wh[:, 1])
    iou = inter / (wh[..., 0] * wh[..., 1] + anchors_wh[:, 0] * anchors_wh[:, 1] - inter)
    return np.argmax(iou, -1)


def encode_one_scale(boxes, classes, num_classes, grid, valid_anchors, anchor_idx=None):
    y = np.zeros((grid, grid, 3, 5 + num_classes), np.float32)
    if len(boxes) == 0:
        return y
    boxes = np.asarray(boxes, np.float32)
    classes = np.asarray(classes, np.int64)
    if anchor_idx is None:
        anchor_idx = find_best_anchor(boxes)
    sel = np.isin(anchor_idx, valid_anchors)
    if not sel.any():
        return y
    b, c, a = boxes[sel], classes[sel], anchor_idx[sel] % 3
    xy = (b[:, 0:2] + b[:, 2:4]) / 2
    wh = b[:, 2:4] - b[:, 0:2]
    cell = np.clip(np.floor(xy / np.float32(1.0 / grid)).astype(np.int64), 0, grid - 1)
    upd = np.zeros((len(b), 5 + num_classes), np.float32)
    upd[:, 0:2], upd[:, 2:4], upd[:, 4] = xy, wh, 1.0
    upd[np.arange(len(b)), 5 + c] = 1.0
    y[cell[:, 1], cell[:, 0], a] = upd
    return y


def encode_labels(boxes, classes, num_classes, grids=GRIDS):
    """Per-scale targets (small, medium, large) for one image."""
    boxes = np.asarray(boxes, np.float32).reshape(-1, 4)
    idx = find_best_anchor(boxes) if len(boxes) else None
    return tuple(encode_one_scale(boxes, classes, num_classes, g, np.array(m), idx)
                 for g, m in zip(grids, ANCHOR_MASKS))


def random_flip(image, boxes, rng):
    """Horizontal flip with probability 0.5 (preprocess.py:44-56); image HWC."""
    if rng.random() < 0.5:
        image = image[:, ::-1]
        boxes = boxes.copy()
        boxes[:, [0, 2]] = 1 - boxes[:, [2, 0]]
    return image, boxes


def random_crop(image, boxes, rng):
    """Crop keeping every box, with probability 0.5 (preprocess.py:58-100)."""
    if rng.random() >= 0.5 or len(boxes) == 0:
        return image, boxes
    x0 = rng.uniform(0, boxes[:, 0].min())
    y0 = rng.uniform(0, boxes[:, 1].min())
    x1 = rng.uniform(0, 1 - boxes[:, 2].max())
    y1 = rng.uniform(0, 1 - boxes[:, 3].max())
    b = boxes.copy()
    b[:, [0, 2]] = (b[:, [0, 2]] - x0) / (1 - x0 - x1)
    b[:, [1, 3]] = (b[:, [1, 3]] - y0) / (1 - y0 - y1)
    h, w = image.shape[:2]
    oy, ox = int(y0 * h), int(x0 * w)
    th, tw = int(np.ceil((1 - y1 - y0) * h)), int(np.ceil((1 - x1 - x0) * w))
    return image[oy:oy + th, ox:ox + tw], b


def synthetic_sample(rng, num_classes=80, size=416, max_boxes=8):
    """Random image in [-1, 1] (CHW float32) and its random ground truth (boxes, classes)."""
    k = int(rng.integers(1, max_boxes + 1))
    c = rng.uniform(0.1, 0.9, (k, 2))
    wh = rng.uniform(0.02, 0.5, (k, 2))
    boxes = np.clip(np.concatenate([c - wh / 2, c + wh / 2], 1), 0.0, 0.999).astype(np.float32)
    classes = rng.integers(0, num_classes, k)
    img = rng.uniform(-1, 1, (3, size, size)).astype(np.float32)
    return img, boxes, classes


# ------------------------------------------------------------------ datasets
def decode_image(encoded: bytes) -> np.ndarray:
    import io

    from PIL import Image

    with Image.open(io.BytesIO(encoded)) as im:
        return np.asarray(im.convert("RGB"))


def resize(image: np.ndarray, size) -> np.ndarray:
    from PIL import Image

    return np.asarray(Image.fromarray(image).resize((size[1], size[0]), Image.BILINEAR))


class YoloTFRecordDataset:
    """COCO / VOC TFRecords (schema of R/Datasets/MSCOCO/tfrecords.py:37-100) -> (image CHW float32 in
    [-1, 1], (y_small, y_medium, y_large)) exactly as Preprocessor.__call__ (preprocess.py:13-35):
    decode, random flip and box-preserving crop when training, resize to 416, /127.5 - 1, encode."""

    def __init__(self, files, is_train, num_classes=80, output_shape=(416, 416), seed=0, encode_on_device=False):
        from .tfrecord import TFRecordIndex

        self.encode_on_device = encode_on_device  # ship padded boxes; ops.labels.yolo_encode on the GPU
        self.index = TFRecordIndex(files)
        self.is_train = is_train
        self.num_classes = num_classes
        self.output_shape = tuple(output_shape)
        self.seed = seed
        self.grids = tuple(output_shape[0] // s for s in (8, 16, 32))

    def __len__(self):
        return len(self.index)

    def __getitem__(self, i):
        from .tfrecord import decode_example, example_values

        ex = decode_example(self.index[i])
        image = decode_image(example_values(ex, "image/encoded")[0])
        classes = np.asarray(example_values(ex, "image/object/class/label", []), np.int64)
        boxes = np.stack([np.asarray(example_values(ex, f"image/object/bbox/{k}", []), np.float32)
                          for k in ("xmin", "ymin", "xmax", "ymax")], 1) if len(classes) else np.zeros((0, 4), np.float32)
        if self.is_train:
            rng = np.random.default_rng((self.seed, i, np.random.randint(1 << 30)))
            image, boxes = random_flip(image, boxes, rng)
            image, boxes = random_crop(image, boxes, rng)
        image = resize(image, self.output_shape).astype(np.float32) / 127.5 - 1
        if self.encode_on_device:
            from ..ops.labels import pad_boxes

            return np.ascontiguousarray(image.transpose(2, 0, 1)), pad_boxes(boxes, classes)
        labels = encode_labels(boxes, classes, self.num_classes, self.grids)
        return np.ascontiguousarray(image.transpose(2, 0, 1)), labels


class SyntheticYoloDataset:
    """Random images + random ground truth of the training shapes (--synthetic)."""

    def __init__(self, n=64, num_classes=80, size=416, seed=0, encode_on_device=False):
        self.n, self.num_classes, self.size, self.seed = n, num_classes, size, seed
        self.grids = tuple(size // s for s in (8, 16, 32))
        self.encode_on_device = encode_on_device

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        rng = np.random.default_rng((self.seed, i))
        img, boxes, classes = synthetic_sample(rng, self.num_classes, self.size)
        if self.encode_on_device:
            from ..ops.labels import pad_boxes

            return img, pad_boxes(boxes, classes)
        return img, encode_labels(boxes, classes, self.num_classes, self.grids)


def collate_raw(batch, grids=GRIDS):
    """Collate of an ``encode_on_device`` dataset: images + {'kind': 'yolo', boxes (N, 100, 4),
    classes (N, 100) int32} for ops.labels.device_targets."""
    import torch

    imgs = torch.from_numpy(np.stack([b[0] for b in batch]))
    boxes = torch.from_numpy(np.stack([b[1][0] for b in batch]))
    classes = torch.from_numpy(np.stack([b[1][1] for b in batch]))
    return imgs, {"kind": "yolo", "boxes": boxes, "classes": classes, "grids": tuple(grids)}


def collate(batch):
    import torch

    imgs = torch.from_numpy(np.stack([b[0] for b in batch]))
    labels = tuple(torch.from_numpy(np.stack([b[1][k] for b in batch])) for k in range(3))
    return imgs, labels
