"""Whole-step deterministic mode (deep_vision_amd.set_deterministic): with it on, the
same training step run twice from the same state gives bitwise-equal losses, gradients, BatchNorm
running statistics and updated weights -- every accumulation on the training path (BN statistics
and backward sums, split-K weight gradients, depthwise / grouped / stem weight gradients, loss
totals) goes through per-block partial rows folded in a fixed order instead of float atomics.

Reference: seeds fixed for reproducibility (R/YOLO/tensorflow/train.py:19); the model shapes are
the reference's families at small batch / resolution."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _build(name):
    from deep_vision_amd import models as M

    torch.manual_seed(0)
    if name == "resnet50":
        return M.ResNet50().to(DEV), (8, 3, 96, 96), "ce"
    if name == "mobilenet1":
        return M.MobileNetV1().to(DEV), (8, 3, 96, 96), "ce"
    if name == "shufflenet1":
        return M.ShuffleNetV1().to(DEV), (8, 3, 96, 96), "ce"
    if name == "inception1":
        return M.InceptionV1().to(DEV), (4, 3, 224, 224), "ce"
    if name == "hourglass":
        return M.StackedHourglassNetwork(num_stack=2, num_residual=1).to(DEV), (4, 3, 128, 128), "hm"
    if name == "yolov3":
        return M.YoloV3(num_classes=20, input_size=128).to(DEV), (2, 3, 128, 128), "yolo"
    raise KeyError(name)


def _loss(out, kind, y):
    from deep_vision_amd import ops as F

    if kind == "ce":
        out = out[0] if isinstance(out, (tuple, list)) else out
        return F.cross_entropy(out, y)
    if kind == "hm":
        from deep_vision_amd.ops.loss import heatmap_mse

        return sum(heatmap_mse(o, y) for o in out)
    from deep_vision_amd.train.detection import yolo_loss

    return yolo_loss(out, y, 20)[0]


def _yolo_labels(n, size, g):
    """One object per image per scale: (N, s, s, 3, 25) with x, y, w, h, obj = 1, a one-hot class."""
    labels = []
    for s in (size // 8, size // 16, size // 32):
        y = torch.zeros(n, s, s, 3, 25, device=DEV)
        for i in range(n):
            cy, cx, a = (int(v) for v in torch.randint(0, s, (2,), generator=g, device=DEV).tolist() + [i % 3])
            y[i, cy, cx, a, :4] = torch.tensor([(cx + 0.5) / s, (cy + 0.5) / s, 0.2, 0.3], device=DEV)
            y[i, cy, cx, a, 4] = 1.0
            y[i, cy, cx, a, 5 + i % 20] = 1.0
        labels.append(y)
    return labels


def _state(m):
    return [t.detach().float().clone() for t in list(m.parameters()) + list(m.buffers()) if t.is_floating_point()]


@pytest.mark.parametrize("name", ["resnet50", "mobilenet1", "shufflenet1", "inception1", "hourglass", "yolov3"])
def test_training_steps_bitwise_reproducible(name):
    from deep_vision_amd import set_deterministic
    from deep_vision_amd.train.optim import FusedSGD

    base, shape, kind = _build(name)
    g = torch.Generator(device=DEV).manual_seed(1)
    xs = [torch.randn(shape, device=DEV, generator=g) for _ in range(2)]
    if kind == "ce":
        ys = [torch.randint(0, 1000, (shape[0],), device=DEV, generator=g) for _ in range(2)]
    elif kind == "hm":
        ys = [torch.rand(shape[0], 16, shape[2] // 4, shape[3] // 4, device=DEV, generator=g) for _ in range(2)]
    else:
        ys = [_yolo_labels(shape[0], shape[2], g) for _ in range(2)]
    runs = []
    set_deterministic(True)
    try:
        for _ in range(2):
            m = copy.deepcopy(base)
            opt = FusedSGD(m.parameters(), lr=1e-3, momentum=0.9, weight_decay=1e-4)
            losses = []
            for i in range(2):
                opt.zero_grad()
                loss = _loss(m(xs[i]), kind, ys[i])
                loss.backward()
                opt.step()
                losses.append(loss.detach().float().clone())
            torch.cuda.synchronize()
            runs.append((torch.stack(losses), _state(m)))
    finally:
        set_deterministic(False)
    (la, sa), (lb, sb) = runs
    assert torch.equal(la, lb), (la.tolist(), lb.tolist())
    bad = [i for i, (a, b) in enumerate(zip(sa, sb)) if not torch.equal(a, b)]
    assert not bad, f"{len(bad)} of {len(sa)} state tensors differ (first index {bad[0]})"


def test_deterministic_flag_roundtrip():
    from deep_vision_amd import set_deterministic
    from deep_vision_amd._ext import lib

    set_deterministic(True)
    assert lib().deterministic()
    set_deterministic(False)
    assert not lib().deterministic()
