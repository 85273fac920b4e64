"""Raw-ground-truth loaders + device target construction (ops.labels) reproduce the host encoders
(data/yolo.py encode_labels, data/pose.py make_heatmaps) exactly: CPU path here, the gfx950
kernels in test_labels_gpu.py."""
import numpy as np
import torch

from deep_vision_amd.data import pose as P
from deep_vision_amd.data import yolo as Y
from deep_vision_amd.ops.labels import device_targets, keypoint_cells, pad_boxes


def test_yolo_raw_collate_matches_host_encoding():
    host = Y.SyntheticYoloDataset(6, 20, 416, seed=3)
    raw = Y.SyntheticYoloDataset(6, 20, 416, seed=3, encode_on_device=True)
    _, ref = Y.collate([host[i] for i in range(6)])
    imgs, r = Y.collate_raw([raw[i] for i in range(6)])
    assert r["boxes"].shape == (6, 100, 4) and r["classes"].dtype == torch.int32
    got = device_targets(r, 20)
    for a, b in zip(got, ref):
        assert torch.equal(a, b)


def test_pose_raw_collate_matches_host_heatmaps():
    host = P.SyntheticPoseDataset(5, 256, (64, 64, 16), seed=4)
    raw = P.SyntheticPoseDataset(5, 256, (64, 64, 16), seed=4, encode_on_device=True)
    ref = torch.stack([torch.from_numpy(host[i][1]) for i in range(5)])
    imgs, r = P.collate_raw([raw[i] for i in range(5)])
    got = device_targets(r, heatmap_shape=(64, 64, 16))
    assert got.shape == ref.shape and torch.equal(got, ref)


def test_pad_boxes_and_cells():
    b, c = pad_boxes(np.array([[0.1, 0.2, 0.3, 0.4]]), np.array([7]), max_boxes=4)
    assert b.shape == (4, 4) and list(c) == [7, -1, -1, -1]
    x, y = keypoint_cells([0.5 / 64 * 3, 2.5 / 64], [1.5 / 64, 0.0], (64, 64, 16))  # halves round to even
    assert list(x) == [2, 2] and list(y) == [2, 0]
