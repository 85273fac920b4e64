"""Inference / export CLI replacing the reference notebooks and scripts.

  classify   top-5 of a classifier checkpoint with ImageNet class names (indices.json /
             synsets.txt); unlike the notebooks (A18) the input IS normalised like training
  detect     YOLOv3: decode + NMS (Postprocessor(iou .5, score .5), demo_mscoco.ipynb)
  pose       Hourglass: keypoints by heatmap argmax with the quarter-pixel shift
  generate   DCGAN samples from the latest checkpoint (R/DCGAN/tensorflow/inference.py)
  translate  CycleGAN A->B / B->A (R/CycleGAN/tensorflow/inference.py)
  export     safetensors weights + a CPU TorchScript trace (the TFLite export of convert.py)

``python -m deep_vision_amd.inference <cmd> ...``; GPU when available (native kernels).
"""
from __future__ import annotations

import argparse
import json
import os

import numpy as np
import torch

from . import models as M
from .train import checkpoint as C


def _device(d=None):
    return torch.device(d or ("cuda" if torch.cuda.is_available() else "cpu"))


def load_model(name, checkpoint=None, key="model", device=None, **kw):
    m = M.get_model(name, **kw)
    if checkpoint:
        ck = C.load(checkpoint)
        sd = ck.get(key, ck) if isinstance(ck, dict) else ck
        m.load_state_dict(C.strip_module_prefix(sd))
    return m.to(_device(device)).eval()


def _load_image(path, size):
    from .data.datasets import load_rgb
    from .data.transforms import CenterCrop, Rescale

    s = {"image": load_rgb(path), "annotation": 0}
    s = CenterCrop(size)(Rescale(int(size * 256 / 224))(s))
    img = s["image"]
    if img.ndim == 2:
        img = np.stack([img] * 3, -1)
    return img


def class_names(path=None):
    if path and path.endswith(".json"):
        with open(path) as f:
            d = json.load(f)
        return {int(k): v for k, v in d.items()}
    if path:
        from .data.datasets import read_synsets

        return read_synsets(path)[1]
    from .data.imagenet_meta import idx_to_name  # packaged ImageNet-2012 names (indices.json)

    return idx_to_name()


@torch.no_grad()
def classify(name, checkpoint, images, names_file=None, topk=5, device=None, size=224):
    from .data.transforms import IMAGENET_MEAN, IMAGENET_STD

    m = load_model(name, checkpoint, device=device)
    names = class_names(names_file)
    out = []
    for p in images:
        img = torch.from_numpy(_load_image(p, size).transpose(2, 0, 1).copy()).float()
        mean = torch.tensor(IMAGENET_MEAN).view(3, 1, 1)
        std = torch.tensor(IMAGENET_STD).view(3, 1, 1)
        x = ((img - mean) / std).unsqueeze(0).to(_device(device))  # 0-255 input, as in training (see transforms)
        prob = torch.softmax(m(x).float(), 1)[0]
        v, i = prob.topk(topk)
        out.append([(int(c), names.get(int(c), str(int(c))), float(s)) for s, c in zip(v.cpu(), i.cpu())])
    return out


@torch.no_grad()
def detect(checkpoint, images, num_classes=80, size=416, iou=0.5, score=0.5, device=None):
    from .data.yolo import resize

    m = load_model("yolov3", checkpoint, device=device, num_classes=num_classes)
    res = []
    for p in images:
        from .data.datasets import load_rgb

        im = load_rgb(p)
        x = torch.from_numpy(resize(im, (size, size)).astype(np.float32) / 127.5 - 1).permute(2, 0, 1)[None]
        boxes, scores, classes, valid = m.detect(x.to(_device(device)), iou, score)
        n = int(valid[0, 0])
        res.append({"boxes": boxes[0, :n].cpu().tolist(), "scores": scores[0, :n, 0].cpu().tolist(),
                    "classes": classes[0, :n].argmax(-1).cpu().tolist()})
    return res


@torch.no_grad()
def pose(checkpoint, images, size=256, num_heatmap=16, device=None):
    from .data.datasets import load_rgb
    from .data.pose import keypoints_from_heatmaps
    from .data.yolo import resize

    m = load_model("hourglass104", checkpoint, device=device, num_heatmap=num_heatmap)
    out = []
    for p in images:
        im = load_rgb(p)
        x = torch.from_numpy(resize(im, (size, size)).astype(np.float32) / 127.5 - 1).permute(2, 0, 1)[None]
        hm = m(x.to(_device(device)))[-1][0].float().cpu().numpy()
        kp = keypoints_from_heatmaps(hm)
        kp[:, 0] *= im.shape[1] / hm.shape[2]
        kp[:, 1] *= im.shape[0] / hm.shape[1]
        out.append(kp.tolist())
    return out


def _save_png(arr, path):
    from PIL import Image

    a = np.clip((arr + 1) * 127.5, 0, 255).astype(np.uint8)
    Image.fromarray(a.squeeze()).save(path)


@torch.no_grad()
def generate(checkpoint_dir="./checkpoints", n=16, out_dir="./generated", device=None, seed=0):
    mgr = C.CheckpointManager(checkpoint_dir)
    g = M.DCGANGenerator().to(_device(device)).eval()
    if mgr.latest_checkpoint:
        g.load_state_dict(C.load(mgr.latest_checkpoint)["generator"])
        print("Restored from {}".format(mgr.latest_checkpoint))
    else:
        print("Initializing from scratch.")
    torch.manual_seed(seed)
    imgs = g(torch.randn(n, 100, device=_device(device))).float().cpu().numpy()
    os.makedirs(out_dir, exist_ok=True)
    paths = []
    for i, im in enumerate(imgs):
        paths.append(os.path.join(out_dir, f"dcgan_{i:03d}.png"))
        _save_png(im[0], paths[-1])
    return paths


@torch.no_grad()
def translate(checkpoint_dir, images, direction="a2b", out_dir="./translated", size=256, device=None):
    from .data.datasets import load_rgb
    from .data.yolo import resize

    mgr = C.CheckpointManager(checkpoint_dir)
    g = M.CycleGANGenerator().to(_device(device)).eval()
    if mgr.latest_checkpoint:
        g.load_state_dict(C.load(mgr.latest_checkpoint)["generator_" + direction])
    os.makedirs(out_dir, exist_ok=True)
    paths = []
    for p in images:
        x = torch.from_numpy(resize(load_rgb(p), (size, size)).astype(np.float32) / 127.5 - 1).permute(2, 0, 1)[None]
        y = g(x.to(_device(device))).float().cpu().numpy()[0].transpose(1, 2, 0)
        paths.append(os.path.join(out_dir, os.path.basename(p) + f".{direction}.png"))
        _save_png(y, paths[-1])
    return paths


def export(name, checkpoint, out_prefix, input_shape=(1, 3, 224, 224), **kw):
    """safetensors weights + TorchScript (traced on CPU through the PyTorch reference path)."""
    from safetensors.torch import save_file

    m = load_model(name, checkpoint, device="cpu", **kw)
    sd = {k: v.contiguous() for k, v in m.state_dict().items()}
    save_file(sd, out_prefix + ".safetensors")
    traced = torch.jit.trace(m, torch.randn(*input_shape), check_trace=False, strict=False)
    traced.save(out_prefix + ".torchscript.pt")
    return out_prefix + ".safetensors", out_prefix + ".torchscript.pt"


def main(argv=None):
    ap = argparse.ArgumentParser(description="deep_vision_amd inference")
    sub = ap.add_subparsers(dest="cmd", required=True)
    c = sub.add_parser("classify")
    c.add_argument("-m", "--model", required=True)
    c.add_argument("-c", "--checkpoint")
    c.add_argument("--names")
    c.add_argument("images", nargs="+")
    d = sub.add_parser("detect")
    d.add_argument("-c", "--checkpoint")
    d.add_argument("--iou", type=float, default=0.5)
    d.add_argument("--score", type=float, default=0.5)
    d.add_argument("images", nargs="+")
    p = sub.add_parser("pose")
    p.add_argument("-c", "--checkpoint")
    p.add_argument("images", nargs="+")
    g = sub.add_parser("generate")
    g.add_argument("--checkpoint-dir", default="./checkpoints")
    g.add_argument("-n", type=int, default=16)
    g.add_argument("--out", default="./generated")
    t = sub.add_parser("translate")
    t.add_argument("--checkpoint-dir", required=True)
    t.add_argument("--direction", default="a2b", choices=["a2b", "b2a"])
    t.add_argument("--out", default="./translated")
    t.add_argument("images", nargs="+")
    e = sub.add_parser("export")
    e.add_argument("-m", "--model", required=True)
    e.add_argument("-c", "--checkpoint")
    e.add_argument("--out", required=True)
    e.add_argument("--size", type=int, default=224)
    a = ap.parse_args(argv)
    if a.cmd == "classify":
        for path, r in zip(a.images, classify(a.model, a.checkpoint, a.images, a.names)):
            print(path, r)
    elif a.cmd == "detect":
        for path, r in zip(a.images, detect(a.checkpoint, a.images, iou=a.iou, score=a.score)):
            print(path, json.dumps(r))
    elif a.cmd == "pose":
        for path, r in zip(a.images, pose(a.checkpoint, a.images)):
            print(path, r)
    elif a.cmd == "generate":
        print(generate(a.checkpoint_dir, a.n, a.out))
    elif a.cmd == "translate":
        print(translate(a.checkpoint_dir, a.images, a.direction, a.out))
    else:
        print(export(a.model, a.checkpoint, a.out, (1, 3, a.size, a.size)))


if __name__ == "__main__":
    main()
