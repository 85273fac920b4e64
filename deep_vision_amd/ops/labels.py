"""Training targets built on the device (csrc/labels.hip).

The loaders can ship raw ground truth instead of encoded targets (``encode_on_device=True`` on
the YOLO / MPII datasets): padded boxes + classes, or integer keypoint coordinates + visibility.
These functions turn a collated batch of that into the exact tensors the host encoders produce
(data/yolo.py ``encode_labels``, data/pose.py ``make_heatmaps``), on the GPU through the native
kernels and on the CPU through the numpy encoders.
"""
from __future__ import annotations

import numpy as np
import torch

from ..models.yolov3 import ANCHORS_WH
from .common import F32, lib, native, ptr, stream_handle

YOLO_GRIDS = (52, 26, 13)


def pad_boxes(boxes, classes, max_boxes=100):
    """One image's (K, 4) boxes / (K,) classes -> fixed-size (max_boxes, 4) float32 and
    (max_boxes,) int32 with class -1 marking padding (the reference keeps <= 100 boxes)."""
    b = np.zeros((max_boxes, 4), np.float32)
    c = np.full((max_boxes,), -1, np.int32)
    k = min(len(classes), max_boxes)
    if k:
        b[:k] = np.asarray(boxes, np.float32).reshape(-1, 4)[:k]
        c[:k] = np.asarray(classes)[:k]
    return b, c


def yolo_encode(boxes: torch.Tensor, classes: torch.Tensor, num_classes: int, grids=YOLO_GRIDS):
    """(N, B, 4) float32 boxes + (N, B) int classes (-1 = padding) -> the three per-scale targets
    (N, g, g, 3, 5 + C) fp32, small grid first."""
    N, B = classes.shape
    D = 5 + num_classes
    if not native(boxes):
        from ..data.yolo import encode_labels

        outs = [[], [], []]
        for n in range(N):
            keep = classes[n] >= 0
            t = encode_labels(boxes[n][keep].cpu().numpy(), classes[n][keep].cpu().numpy(), num_classes, grids)
            for k in range(3):
                outs[k].append(torch.from_numpy(t[k]))
        return tuple(torch.stack(o).to(boxes.device) for o in outs)
    boxes = boxes.to(F32).contiguous()
    classes = classes.to(torch.int32).contiguous()
    ys = [torch.zeros((N, g, g, 3, D), dtype=F32, device=boxes.device) for g in grids]
    lib().yolo_encode(ptr(boxes), ptr(classes), N, B, num_classes, [float(v) for v in ANCHORS_WH.reshape(-1)],
                      ptr(ys[0]), ptr(ys[1]), ptr(ys[2]), grids[0], grids[1], grids[2], stream_handle())
    return tuple(ys)


def keypoint_cells(kx, ky, shape=(64, 64, 16)):
    """Host-side integer heatmap coordinates, rounded half-to-even exactly as make_heatmaps does."""
    x = np.round(np.asarray(kx) * shape[0]).astype(np.int32)
    y = np.round(np.asarray(ky) * shape[1]).astype(np.int32)
    return x, y


def render_heatmaps(px: torch.Tensor, py: torch.Tensor, vis: torch.Tensor, shape=(64, 64, 16)) -> torch.Tensor:
    """(N, J) integer keypoint cells + visibility -> (N, J, H, W) fp32 Gaussian targets (sigma 1,
    7x7 window, peak 12), H = shape[1], W = shape[0]."""
    N, J = px.shape
    H, W = shape[1], shape[0]
    if not native(px):
        from ..data.pose import gaussian_heatmap

        out = np.zeros((N, J, H, W), np.float32)
        for n in range(N):
            for j in range(J):
                out[n, j] = gaussian_heatmap(H, W, int(py[n, j]), int(px[n, j]), int(vis[n, j]))
        return torch.from_numpy(out).to(px.device)
    px, py, vis = (t.to(torch.int32).contiguous() for t in (px, py, vis))
    out = torch.empty((N, J, H, W), dtype=F32, device=px.device)
    lib().heatmaps(ptr(px), ptr(py), ptr(vis), N, J, H, W, ptr(out), stream_handle())
    return out


def device_targets(raw, num_classes=80, heatmap_shape=(64, 64, 16)):
    """A collated raw-ground-truth batch (data.yolo.collate_raw / data.pose.collate_raw), already on
    the training device -> the encoded targets the losses consume."""
    kind = raw["kind"]
    if kind == "yolo":
        return yolo_encode(raw["boxes"], raw["classes"], num_classes, tuple(raw.get("grids", YOLO_GRIDS)))
    if kind == "pose":
        return render_heatmaps(raw["px"], raw["py"], raw["vis"], heatmap_shape)
    raise ValueError(f"unknown raw target kind {kind!r}")
