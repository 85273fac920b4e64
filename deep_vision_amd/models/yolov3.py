"""YOLOv3 with a Darknet-53 backbone (R/YOLO/tensorflow/yolov3.py:20-205).

Keras semantics are kept where they change numerics or parameters:
  * every DarknetConv is Conv2D('same', no bias) -> BatchNormalization (eps 1e-3, Keras momentum
    0.99 = torch momentum 0.01) -> LeakyReLU(0.1); the stride-2 'same' convs pad 0 top/left and
    1 bottom/right, which the native conv takes as an asymmetric pad (no padded copy);
  * heads are 1x1 Conv2D with bias producing 3*(5+C) channels, viewed as (N, g, g, 3, 5+C) --
    a free view of the NHWC conv output (the channel row stride may be padded to a multiple of 8).
Module names follow the Keras layer names (``conv2d_0``, ``residual_2_7``,
``detector_scale_large_1x1_1`` ...), giving 61,949,149 trainable parameters for 80 classes
(pinned in tests).

``forward`` returns the three raw head tensors (small 52x52, medium 26x26, large 13x13 for a
416 input) in training mode, as ``YoloV3(training=True)``; ``decode()`` / ``detect()`` give the
inference outputs (absolute boxes, NMS).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as tnn

from .. import nn
from .. import ops as F
from ..ops.conv import GradJoin

# R/YOLO/tensorflow/yolov3.py:19-21
ANCHORS_WH = np.array([[10, 13], [16, 30], [33, 23], [30, 61], [62, 45], [59, 119], [116, 90], [156, 198],
                       [373, 326]], np.float32) / 416
ANCHOR_MASKS = ((0, 1, 2), (3, 4, 5), (6, 7, 8))  # small, medium, large scale


class DarknetConv(tnn.Module):
    def __init__(self, cin, cout, k, stride):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, k, stride=stride, padding="same_keras", bias=False)
        self.bn = nn.BatchNorm2d(cout, eps=1e-3, momentum=0.01)

    def forward(self, x, residual=None, join=None, join_role=None, residual_join=None):
        # residual: out = leaky(bn(conv(x))) + residual, the add inside the BN apply pass
        return F.conv_bn_act(x, self.conv, self.bn, "leaky", 0.1, residual=residual, residual_post=True, join=join,
                             join_role=join_role, residual_join=residual_join)


class DarknetResidual(tnn.Module):
    def __init__(self, c1, c2):
        super().__init__()
        self.conv_1x1 = DarknetConv(c2, c1, 1, 1)
        self.conv_3x3 = DarknetConv(c1, c2, 3, 1)

    def forward(self, x):
        # Add()([shortcut, LeakyReLU(BN(conv))]): the add follows the activation and rides in the
        # BN apply pass; x's two gradients (the shortcut's = the block output's gradient, and
        # conv_1x1's input gradient) meet in conv_1x1's dgrad epilogue (ops.conv.GradJoin)
        # instead of an autograd add
        j = GradJoin() if F.native(x) else None
        y = self.conv_1x1(x, join=j, join_role="consumer")
        return self.conv_3x3(y, residual=x, residual_join=j)


class Darknet53(tnn.Module):
    """R/YOLO/tensorflow/yolov3.py:62-92: returns the stride-8/16/32 feature maps."""

    STAGES = ((64, 32, 1), (128, 64, 2), (256, 128, 8), (512, 256, 8), (1024, 512, 4))

    def __init__(self):
        super().__init__()
        self.conv2d_0 = DarknetConv(3, 32, 3, 1)
        cin = 32
        for i, (cout, mid, n) in enumerate(self.STAGES):
            setattr(self, f"conv2d_{i + 1}", DarknetConv(cin, cout, 3, 2))
            setattr(self, f"residual_{i}", tnn.Sequential(*[DarknetResidual(mid, cout) for _ in range(n)]))
            cin = cout

    def forward(self, x):
        x = self.conv2d_0(x)
        outs = []
        for i in range(5):
            x = getattr(self, f"residual_{i}")(getattr(self, f"conv2d_{i + 1}")(x))
            if i >= 2:
                outs.append(x)
        return tuple(outs)


class _DetectorScale(tnn.Module):
    """1x1/3x3 x3 detector block of one scale + the final 1x1 conv (yolov3.py:104-190)."""

    def __init__(self, cin, c, final):
        super().__init__()
        self.c1x1_1 = DarknetConv(cin, c, 1, 1)
        self.c3x3_1 = DarknetConv(c, 2 * c, 3, 1)
        self.c1x1_2 = DarknetConv(2 * c, c, 1, 1)
        self.c3x3_2 = DarknetConv(c, 2 * c, 3, 1)
        self.c1x1_3 = DarknetConv(2 * c, c, 1, 1)
        self.c3x3_3 = DarknetConv(c, 2 * c, 3, 1)
        self.final_conv2d = nn.Conv2d(2 * c, final, 1)

    def forward(self, x):
        x = self.c1x1_3(self.c3x3_2(self.c1x1_2(self.c3x3_1(self.c1x1_1(x)))))
        return x, self.final_conv2d(self.c3x3_3(x))


def _head_view(y):
    """(N, 3*(5+C), g, g) conv output -> (N, g, g, 3, 5+C) (free view of the NHWC rows)."""
    N, ch, g, g2 = y.shape
    return y.permute(0, 2, 3, 1).unflatten(3, (3, ch // 3))


class YoloV3(tnn.Module):
    def __init__(self, num_classes=80, input_size=416):
        super().__init__()
        self.num_classes = num_classes
        self.input_size = input_size
        final = 3 * (5 + num_classes)
        self.backbone = Darknet53()
        self.detector_scale_large = _DetectorScale(1024, 512, final)
        self.detector_scale_medium_1x1_0 = DarknetConv(512, 256, 1, 1)
        self.detector_scale_medium = _DetectorScale(256 + 512, 256, final)
        self.detector_scale_small_1x1_0 = DarknetConv(256, 128, 1, 1)
        self.detector_scale_small = _DetectorScale(128 + 256, 128, final)

    @staticmethod
    def _up_cat(x, skip):
        return F.concat([F.upsample_nearest(x, 2), skip])  # route (yolov3.py:151-152,180-181)

    def forward(self, x):
        """Raw head tensors (small, medium, large), each (N, g, g, 3, 5+C)."""
        x_small, x_medium, x_large = self.backbone(x)
        x, y_large = self.detector_scale_large(x_large)
        x = self._up_cat(self.detector_scale_medium_1x1_0(x), x_medium)
        x, y_medium = self.detector_scale_medium(x)
        x = self._up_cat(self.detector_scale_small_1x1_0(x), x_small)
        x, y_small = self.detector_scale_small(x)
        return _head_view(y_small), _head_view(y_medium), _head_view(y_large)

    def decode(self, heads):
        """Absolute boxes of all scales: (N, sum 3*g*g, 5+C) rows [x1, y1, x2, y2, obj, class probs]
        (get_absolute_yolo_box + xywh_to_x1x2y1y2, yolov3.py:208-231, postprocess.py:16-27)."""
        from ..ops.detection import yolo_decode

        return yolo_decode(heads, [ANCHORS_WH[list(m)] for m in ANCHOR_MASKS])

    @torch.no_grad()
    def detect(self, x, iou_thresh=0.5, score_thresh=0.5, max_detection=100):
        """Postprocessor(iou_thresh, score_thresh, max_detection)(model(x)) of the reference:
        returns boxes (N, 100, 4), scores (N, 100, 1), class probs (N, 100, C), valid (N, 1)."""
        from ..ops.detection import batch_nms

        return batch_nms(self.decode(self.forward(x)), iou_thresh, score_thresh, max_detection)
