"""Detection-head ops: YOLOv3 loss, box decode, greedy NMS, box utilities.

GPU tensors run the fused kernels of csrc/yolo.hip; CPU tensors run the plain PyTorch versions
below, which also serve as the numerics oracle in tests/test_detection*.py.

Reference semantics: R/YOLO/tensorflow/yolov3.py:208-371 (get_absolute_yolo_box,
get_relative_yolo_box, YoloLoss), utils.py (xywh_to_x1x2y1y2, xywh_to_y1x1y2x2, broadcast_iou,
binary_cross_entropy), postprocess.py (Postprocessor.batch_non_maximum_suppression).
"""
from __future__ import annotations

import torch

from .common import BF16, F32, lib, native, ptr, stream_handle

MAX_GT = 100  # ground-truth boxes considered by the ignore mask (yolov3.py:293)


# ----------------------------------- box utilities -----------------------------------
def xywh_to_x1x2y1y2(box):
    """(cx, cy, w, h) -> (x1, y1, x2, y2) (the reference's name, its output order is x1y1x2y2)."""
    xy, wh = box[..., 0:2], box[..., 2:4]
    return torch.cat([xy - wh / 2, xy + wh / 2], -1)


def xywh_to_y1x1y2x2(box):
    x, y, w, h = box[..., 0:1], box[..., 1:2], box[..., 2:3], box[..., 3:4]
    yx, hw = torch.cat([y, x], -1), torch.cat([h, w], -1)
    return torch.cat([yx - hw / 2, yx + hw / 2], -1)


def broadcast_iou(box_a, box_b):
    """IoU of (..., N, 4) against (..., M, 4) x1y1x2y2 boxes -> (..., N, M); intersection sides
    clipped to [0, 1] and union + 1e-7 as in the reference (utils.py broadcast_iou)."""
    a = box_a.unsqueeze(-2)
    b = box_b.unsqueeze(-3)
    iw = (torch.minimum(a[..., 2], b[..., 2]) - torch.maximum(a[..., 0], b[..., 0])).clamp(0, 1)
    ih = (torch.minimum(a[..., 3], b[..., 3]) - torch.maximum(a[..., 1], b[..., 1])).clamp(0, 1)
    i = iw * ih
    area_a = (a[..., 2] - a[..., 0]) * (a[..., 3] - a[..., 1])
    area_b = (b[..., 2] - b[..., 0]) * (b[..., 3] - b[..., 1])
    return i / (area_a + area_b - i + 1e-7)


def binary_cross_entropy(probs, labels, eps=1e-7):
    p = probs.clamp(eps, 1 - eps)
    return -(labels * torch.log(p) + (1 - labels) * torch.log(1 - p))


def _grid(g, device):
    gy, gx = torch.meshgrid(torch.arange(g, device=device), torch.arange(g, device=device), indexing="ij")
    return torch.stack([gx, gy], -1).unsqueeze(2).float()  # (g, g, 1, 2) = (x, y)


def get_absolute_yolo_box(y_pred, anchors_wh, num_classes):
    """Raw head (N, g, g, 3, 5+C) -> box (cx, cy, w, h), objectness, class probs (yolov3.py:208)."""
    y_pred = y_pred.float()
    t_xy, t_wh, obj, cls = torch.split(y_pred, (2, 2, 1, num_classes), -1)
    g = y_pred.shape[1]
    anchors = torch.as_tensor(anchors_wh, dtype=F32, device=y_pred.device)
    b_xy = (torch.sigmoid(t_xy) + _grid(g, y_pred.device)) / g
    b_wh = torch.exp(t_wh) * anchors
    return torch.cat([b_xy, b_wh], -1), torch.sigmoid(obj), torch.sigmoid(cls)


def get_relative_yolo_box(y_true, anchors_wh):
    """Inverse of get_absolute_yolo_box for the ground truth (yolov3.py:234-256)."""
    g = y_true.shape[1]
    anchors = torch.as_tensor(anchors_wh, dtype=F32, device=y_true.device)
    t_xy = y_true[..., 0:2] * g - _grid(g, y_true.device)
    t_wh = torch.log(y_true[..., 2:4] / anchors)
    t_wh = torch.where(torch.isfinite(t_wh), t_wh, torch.zeros_like(t_wh))
    return torch.cat([t_xy, t_wh], -1)


def _gt_boxes(y_true):
    """First MAX_GT ground-truth boxes (cell order) per image, x1y1x2y2, zero-padded: (N, 100, 4)."""
    N = y_true.shape[0]
    flat = y_true.reshape(N, -1, y_true.shape[-1])
    out = torch.zeros((N, MAX_GT, 4), dtype=F32, device=y_true.device)
    for n in range(N):
        rows = flat[n][flat[n, :, 4] > 0][:MAX_GT]
        out[n, : rows.shape[0]] = xywh_to_x1x2y1y2(rows[:, :4].float())
    return out


def yolo_loss_torch(y_pred, y_true, anchors_wh, num_classes, lambda_coord=5.0, lambda_noobj=0.5, ignore_thresh=0.5):
    """Per-image loss components (N, 4) = (xy, wh, class, obj) of one scale, autograd-able."""
    y_pred = y_pred.float()
    y_true = y_true.float()
    pred_xy_rel = torch.sigmoid(y_pred[..., 0:2])
    pred_wh_rel = y_pred[..., 2:4]
    box_abs, pred_obj, pred_cls = get_absolute_yolo_box(y_pred, anchors_wh, num_classes)
    pred_box = xywh_to_x1x2y1y2(box_abs)
    true_xywh, true_obj, true_cls = y_true[..., 0:4], y_true[..., 4:5], y_true[..., 5:]
    rel = get_relative_yolo_box(y_true, anchors_wh)
    weight = 2 - true_xywh[..., 2] * true_xywh[..., 3]
    tobj = true_obj[..., 0]
    xy = (((rel[..., 0:2] - pred_xy_rel) ** 2).sum(-1) * tobj * weight).sum((1, 2, 3)) * lambda_coord
    wh = (((rel[..., 2:4] - pred_wh_rel) ** 2).sum(-1) * tobj * weight).sum((1, 2, 3)) * lambda_coord
    cls = (binary_cross_entropy(pred_cls, true_cls) * true_obj).sum((1, 2, 3, 4))
    N = y_pred.shape[0]
    with torch.no_grad():
        best = broadcast_iou(pred_box.reshape(N, -1, 4), _gt_boxes(y_true)).amax(-1)
        ignore = (best < ignore_thresh).float().reshape(tobj.shape).unsqueeze(-1)
    ent = binary_cross_entropy(pred_obj, true_obj)
    obj = (true_obj * ent).sum((1, 2, 3, 4)) + ((1 - true_obj) * ent * ignore).sum((1, 2, 3, 4)) * lambda_noobj
    return torch.stack([xy, wh, cls, obj], 1)


def _head_geometry(y_pred):
    N, g, g2, A, D = y_pred.shape
    ldp = y_pred.stride(2)
    ok = (A == 3 and g == g2 and y_pred.dtype == BF16 and y_pred.stride(4) == 1 and y_pred.stride(3) == D
          and ldp >= 3 * D and y_pred.stride(1) == g * ldp and y_pred.stride(0) == g * g * ldp)
    return ok, N, g, D, ldp


class _YoloLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y_pred, y_true, anchors, num_classes, lambda_coord, lambda_noobj, ignore_thresh):
        ok, N, g, D, ldp = _head_geometry(y_pred)
        dev = y_pred.device
        boxes = torch.zeros((N, MAX_GT, 4), dtype=F32, device=dev)
        counts = torch.empty(N, dtype=torch.int32, device=dev)
        st = stream_handle()
        lib().yolo_gather_boxes(ptr(y_true), N, g * g * 3, D, ptr(boxes), ptr(counts), st)
        losses = torch.zeros((N, 4), dtype=F32, device=dev)
        cfg = (N, g, num_classes, anchors, lambda_coord, lambda_noobj, ignore_thresh, ldp)
        lib().yolo_loss(ptr(y_pred), ldp, ptr(y_true), ptr(boxes), ptr(counts), 0, 0, ptr(losses), N, g, num_classes,
                        list(anchors), 1.0, lambda_coord, lambda_noobj, ignore_thresh, st)
        ctx.save_for_backward(y_pred, y_true, boxes, counts)
        ctx.cfg = cfg
        return losses

    @staticmethod
    def backward(ctx, gout):
        y_pred, y_true, boxes, counts = ctx.saved_tensors
        N, g, C, anchors, lc, ln, it, ldp = ctx.cfg
        D = 5 + C
        gw = gout.float().contiguous()
        full = torch.empty((N, g, g, ldp), dtype=BF16, device=y_pred.device)
        lib().yolo_loss(ptr(y_pred), ldp, ptr(y_true), ptr(boxes), ptr(counts), ptr(full), ptr(gw), 0, N, g, C,
                        list(anchors), 1.0, lc, ln, it, stream_handle())
        grad = full[..., : 3 * D].unflatten(3, (3, D))
        return grad, None, None, None, None, None, None


def yolo_loss(y_pred, y_true, anchors_wh, num_classes, lambda_coord=5.0, lambda_noobj=0.5, ignore_thresh=0.5):
    """YoloLoss of one scale: (N, 4) per-image components (xy, wh, class, obj); the reference's
    total is ``.sum(1)``. ``y_pred`` is the raw (N, g, g, 3, 5+C) head, ``y_true`` the encoded
    label of that scale (deep_vision_amd.data.yolo.encode_labels)."""
    anchors = tuple(float(v) for v in torch.as_tensor(anchors_wh, dtype=F32).reshape(-1).tolist())
    if native(y_pred):
        ok = _head_geometry(y_pred)[0]
        if not ok:
            raise ValueError("yolo_loss expects the bf16 (N, g, g, 3, 5+C) view of a head conv output")
        y_true = y_true.to(device=y_pred.device, dtype=F32).contiguous()
        return _YoloLossFn.apply(y_pred, y_true, anchors, int(num_classes), float(lambda_coord),
                                 float(lambda_noobj), float(ignore_thresh))
    return yolo_loss_torch(y_pred, y_true, torch.tensor(anchors).view(3, 2), num_classes, lambda_coord,
                           lambda_noobj, ignore_thresh)


# ----------------------------------- decode + NMS -----------------------------------
def yolo_decode(heads, anchors_per_scale):
    """Concatenated absolute detections of all scales: (N, M, 5+C) rows
    [x1, y1, x2, y2, objectness, class probs] (row order: scale, cell, anchor)."""
    N = heads[0].shape[0]
    D = heads[0].shape[-1]
    C = D - 5
    M = sum(h.shape[1] * h.shape[2] * 3 for h in heads)
    if native(heads[0]) and all(_head_geometry(h)[0] for h in heads):
        out = torch.empty((N, M, D), dtype=F32, device=heads[0].device)
        off = 0
        for h, anc in zip(heads, anchors_per_scale):
            _, _, g, _, ldp = _head_geometry(h)
            lib().yolo_decode(ptr(h), ldp, N, g, C, [float(v) for v in torch.as_tensor(anc).reshape(-1).tolist()],
                              ptr(out), M, off, stream_handle())
            off += g * g * 3
        return out
    rows = []
    for h, anc in zip(heads, anchors_per_scale):
        box, obj, cls = get_absolute_yolo_box(h, anc, C)
        rows.append(torch.cat([xywh_to_x1x2y1y2(box), obj, cls], -1).reshape(N, -1, D))
    return torch.cat(rows, 1)


def _nms_torch(cand, iou_thresh, score_thresh, max_det):
    N, M, D = cand.shape
    out = torch.zeros((N, max_det + 1, D), dtype=F32, device=cand.device)
    for n in range(N):
        c = cand[n][cand[n, :, 4] >= score_thresh]
        count = 0
        while c.shape[0] > 0 and count < max_det:
            i = int(torch.argmax(c[:, 4]))
            best = c[i]
            out[n, count] = best
            count += 1
            c = torch.cat([c[:i], c[i + 1:]], 0)
            iou = broadcast_iou(best[None, :4], c[:, :4])[0]
            c = c[iou <= iou_thresh]
        if count:
            out[n, max_det] = count
    return out


def batch_nms(cand, iou_thresh=0.5, score_thresh=0.5, max_detection=100):
    """Multi-label greedy NMS (postprocess.py:31-95) on (N, M, 5+C) decoded rows.

    Returns (boxes (N, K, 4), scores (N, K, 1), class probs (N, K, C), valid (N, 1) int32)
    with K = max_detection, zero rows past ``valid``."""
    cand = cand.float().contiguous()
    N, M, D = cand.shape
    if native(cand):
        out = torch.zeros((N, max_detection + 1, D), dtype=F32, device=cand.device)
        lib().nms(ptr(cand), N, M, D, float(iou_thresh), float(score_thresh), int(max_detection), ptr(out),
                  stream_handle())
    else:
        out = _nms_torch(cand, iou_thresh, score_thresh, max_detection)
    valid = out[:, max_detection, 0:1].to(torch.int32)
    res = out[:, :max_detection]
    return res[..., 0:4], res[..., 4:5], res[..., 5:], valid
