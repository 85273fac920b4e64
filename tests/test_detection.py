"""CPU semantics of the detection / GAN building blocks (the GPU kernels are compared against these
in tests/test_heads_gpu.py).

* Keras 'same' conv / Conv2DTranspose geometry against a direct definition
* YOLO label encoding (best anchor by wh-IoU, cell of the centre) -- R/YOLO/tensorflow/preprocess.py
* YOLO loss: zero box/class loss at the exact target, ignore mask, component structure
* greedy NMS against a brute-force re-implementation of postprocess.py's loop
"""
import numpy as np
import pytest
import torch

from deep_vision_amd import nn
from deep_vision_amd.data import yolo as Y
from deep_vision_amd.models.yolov3 import ANCHORS_WH
from deep_vision_amd.ops import detection as D


def test_keras_same_conv_padding():
    conv = nn.Conv2d(4, 6, 3, stride=2, padding="same_keras")
    assert conv.native_padding(8, 8) == (0, 1, 0, 1)  # extra row/col at the bottom/right
    assert conv.native_padding(7, 7) == (1, 1)
    x = torch.randn(2, 4, 8, 8)
    ref = torch.nn.functional.conv2d(torch.nn.functional.pad(x, (0, 1, 0, 1)), conv.weight, conv.bias, 2)
    assert torch.allclose(conv(x), ref, atol=1e-6)
    assert nn.Conv2d(3, 8, 7, stride=2, padding="same_keras").native_padding(256, 256) == (2, 3, 2, 3)


@pytest.mark.parametrize("k,s,H", [(5, 2, 7), (5, 1, 7), (3, 2, 5), (4, 2, 6)])
def test_keras_same_conv_transpose(k, s, H):
    ct = nn.ConvTranspose2d(3, 2, k, stride=s, padding="same_keras", bias=False)
    x = torch.randn(1, 3, H, H)
    y = ct(x)
    assert y.shape == (1, 2, H * s, H * s)
    # direct definition: y[o] += x[i] w[r] with o = i*s - pad + r, pad = (k - s) // 2
    pad = max(k - s, 0) // 2
    ref = torch.zeros(1, 2, H * s, H * s)
    w = ct.weight.detach()
    for i in range(H):
        for j in range(H):
            for r in range(k):
                for c in range(k):
                    o, q = i * s - pad + r, j * s - pad + c
                    if 0 <= o < H * s and 0 <= q < H * s:
                        ref[0, :, o, q] += torch.einsum("i,io->o", x[0, :, i, j], w[:, :, r, c])
    assert torch.allclose(y, ref, atol=1e-5)


def test_yolo_label_encoding():
    boxes = np.array([[0.1, 0.1, 0.13, 0.14], [0.3, 0.3, 0.9, 0.95]], np.float32)
    classes = np.array([3, 7])
    small, medium, large = Y.encode_labels(boxes, classes, 80)
    assert small.shape == (52, 52, 3, 85) and large.shape == (13, 13, 3, 85)
    a = Y.find_best_anchor(boxes)
    assert a[0] in (0, 1, 2) and a[1] in (6, 7, 8)
    cx, cy = 0.115, 0.12
    row = small[int(cy * 52), int(cx * 52), a[0] % 3]
    assert np.allclose(row[:4], [cx, cy, 0.03, 0.04], atol=1e-6) and row[4] == 1 and row[5 + 3] == 1
    assert small[..., 4].sum() == 1 and medium[..., 4].sum() == 0 and large[..., 4].sum() == 1


def _random_targets(N, C=80, seed=0):
    rng = np.random.default_rng(seed)
    ys = [[], [], []]
    for _ in range(N):
        _, b, c = Y.synthetic_sample(rng, C, size=8)
        for k, t in enumerate(Y.encode_labels(b, c, C)):
            ys[k].append(t)
    return [torch.from_numpy(np.stack(t)) for t in ys]


def test_yolo_loss_structure_and_exact_target():
    torch.manual_seed(0)
    C = 80
    y_true = _random_targets(2, C)[0]  # 52x52 scale
    anchors = ANCHORS_WH[0:3]
    pred = torch.randn(2, 52, 52, 3, 5 + C, requires_grad=True)
    comp = D.yolo_loss(pred, y_true, anchors, C)
    assert comp.shape == (2, 4) and torch.all(comp >= 0)
    comp.sum().backward()
    assert torch.isfinite(pred.grad).all()
    # predictions equal to the encoded targets give zero xy/wh loss
    rel = D.get_relative_yolo_box(y_true, anchors)
    p = torch.zeros_like(pred)
    p[..., 0:2] = torch.logit(rel[..., 0:2].clamp(1e-6, 1 - 1e-6))
    p[..., 2:4] = rel[..., 2:4]
    p[..., 4:] = torch.where(y_true[..., 4:] > 0, 30.0, -30.0)
    comp = D.yolo_loss(p, y_true, anchors, C)
    assert comp[:, 0].abs().max() < 1e-4 and comp[:, 1].abs().max() < 1e-6
    assert comp[:, 2].max() < 1e-3  # BCE clipped at 1e-7


def _brute_nms(cand, iou_t, score_t, max_det):
    out = []
    for n in range(cand.shape[0]):
        c = [r for r in cand[n].tolist() if r[4] >= score_t]
        keep = []
        while c and len(keep) < max_det:
            i = max(range(len(c)), key=lambda j: (c[j][4], -j))
            b = c.pop(i)
            keep.append(b)
            bt = torch.tensor([b[:4]])
            c = [r for r in c if D.broadcast_iou(bt, torch.tensor([r[:4]]))[0, 0] <= iou_t]
        out.append(keep)
    return out


def test_nms_matches_reference_loop():
    torch.manual_seed(1)
    N, M, C = 2, 60, 3
    xy = torch.rand(N, M, 2) * 0.8
    wh = torch.rand(N, M, 2) * 0.3 + 0.05
    cand = torch.cat([xy, xy + wh, torch.rand(N, M, 1), torch.rand(N, M, C)], -1)
    boxes, scores, classes, valid = D.batch_nms(cand, 0.4, 0.3, 10)
    ref = _brute_nms(cand, 0.4, 0.3, 10)
    for n in range(N):
        k = len(ref[n])
        assert valid[n, 0] == k
        got = torch.cat([boxes[n, :k], scores[n, :k], classes[n, :k]], -1)
        assert torch.allclose(got, torch.tensor(ref[n]), atol=1e-6)
        assert torch.all(boxes[n, k:] == 0)


def test_yolov3_decode_shapes():
    from deep_vision_amd.models.yolov3 import YoloV3

    m = YoloV3(num_classes=4).eval()
    with torch.no_grad():
        heads = m(torch.randn(1, 3, 64, 64))
        cand = m.decode(heads)
    assert cand.shape == (1, (8 * 8 + 4 * 4 + 2 * 2) * 3, 9)
    assert torch.all(cand[..., 4:] >= 0) and torch.all(cand[..., 4:] <= 1)
    b, s, c, v = D.batch_nms(cand, 0.5, 0.0, 100)
    assert b.shape == (1, 100, 4) and c.shape == (1, 100, 4) and v.shape == (1, 1)


def test_pointwise_losses_cpu():
    from deep_vision_amd.ops import loss as L

    p = torch.randn(2, 16, 8, 8)
    t = torch.rand(2, 16, 8, 8) * (torch.rand(2, 16, 8, 8) > 0.8)
    w = (t > 0).float() * 81 + 1
    assert torch.allclose(L.heatmap_mse(p, t), ((t - p) ** 2 * w).mean())
    assert torch.allclose(L.bce_with_logits(p, 1.0), torch.nn.functional.softplus(-p).mean(), atol=1e-6)
    assert torch.allclose(L.mse_loss(p, 0.0), (p ** 2).mean())
    assert torch.allclose(L.l1_loss(p, t), (p - t).abs().mean())
    assert torch.isfinite(L.focal_loss(p, t))
