"""gfx950 target-construction kernels (csrc/labels.hip) against the host numpy encoders: YOLO
3-scale label encoding (best anchor, grid cell, last-box-wins on shared cells) and the Hourglass
Gaussian heatmaps (window clipping at every border, invisible joints)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _ext():
    from deep_vision_amd._ext import lib

    lib()


def test_yolo_encode_kernel_matches_numpy():
    from deep_vision_amd.data.yolo import encode_labels
    from deep_vision_amd.ops.labels import pad_boxes, yolo_encode

    rng = np.random.default_rng(0)
    N, C = 16, 80
    bs, cs, ref = [], [], [[], [], []]
    for n in range(N):
        k = int(rng.integers(0, 60))
        xy = rng.uniform(0, 1, (k, 2))
        wh = rng.uniform(0.005, 0.9, (k, 2))
        boxes = np.clip(np.concatenate([xy - wh / 2, xy + wh / 2], 1), 0, 1).astype(np.float32)
        if k > 3:  # duplicates: identical boxes with different classes land on one (cell, anchor)
            boxes[1] = boxes[0]
        cls = rng.integers(0, C, k)
        t = encode_labels(boxes, cls, C)
        for s in range(3):
            ref[s].append(t[s])
        b, c = pad_boxes(boxes, cls)
        bs.append(b)
        cs.append(c)
    got = yolo_encode(torch.from_numpy(np.stack(bs)).cuda(), torch.from_numpy(np.stack(cs)).cuda(), C)
    for s in range(3):
        r = torch.from_numpy(np.stack(ref[s]))
        assert got[s].shape == r.shape
        assert torch.equal(got[s].cpu(), r), (s, (got[s].cpu() - r).abs().max())


def test_heatmap_kernel_matches_numpy():
    from deep_vision_amd.data.pose import make_heatmaps
    from deep_vision_amd.ops.labels import keypoint_cells, render_heatmaps

    rng = np.random.default_rng(1)
    N, J = 12, 16
    kx = rng.uniform(-0.1, 1.1, (N, J))  # off-map and border keypoints included
    ky = rng.uniform(-0.1, 1.1, (N, J))
    v = rng.integers(0, 3, (N, J))
    ref = np.stack([make_heatmaps(kx[n], ky[n], v[n], (64, 64, J)).transpose(2, 0, 1) for n in range(N)])
    px, py = keypoint_cells(kx, ky, (64, 64, J))
    got = render_heatmaps(torch.from_numpy(px).cuda(), torch.from_numpy(py).cuda(), torch.from_numpy(v).cuda(),
                          (64, 64, J))
    assert got.shape == ref.shape
    np.testing.assert_allclose(got.cpu().numpy(), ref, rtol=1e-6, atol=0)
