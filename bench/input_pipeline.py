#!/usr/bin/env python3
"""Input-pipeline throughput: decode + augment images/s per loader worker on
JPEGs generated locally with PIL (no dataset download), for the reference pipeline (float CHW,
normalised on the host: R/ResNet/pytorch/data_load.py:72-297, R/ResNet/pytorch/train.py:315-331)
and the device-normalised one (uint8 HWC crops, data/device_input.py), plus DataLoader rates at
several worker counts and -- on a GPU -- the H2D + device normalise cost per batch.

    python bench/input_pipeline.py [--images 256] [--workers 1,2,4,8] [--batch 256] [--out FILE]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def make_jpegs(d, n, seed=0):
    """ImageNet-like JPEGs: ~500x375 average, photo-like smooth content + noise, quality 90,
    flattened-train naming (nXXXXXXXX_<i>.JPEG) so ImageNet2012Dataset reads them."""
    import numpy as np
    from PIL import Image

    rng = np.random.RandomState(seed)
    syn = [f"n{1440764 + k:08d}" for k in range(10)]
    for i in range(n):
        h, w = int(rng.randint(300, 450)), int(rng.randint(400, 600))
        yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
        base = np.stack([np.sin(xx / rng.uniform(20, 80) + c) * np.cos(yy / rng.uniform(20, 80)) for c in range(3)], -1)
        img = ((base * 0.5 + 0.5) * 200 + rng.normal(0, 12, (h, w, 3))).clip(0, 255).astype(np.uint8)
        Image.fromarray(img).save(os.path.join(d, f"{syn[i % 10]}_{i}.JPEG"), quality=90)
    path = os.path.join(os.path.dirname(d), "synsets.txt")  # beside the flattened dir, not in it
    with open(path, "w") as f:
        for s in syn:
            f.write(f"{s} class_{s}\n")
    return path


def per_worker_rate(ds, n):
    ds[0]  # first-use imports (pyarrow for the zero-copy decode) stay out of the timing, as in a worker
    t0 = time.perf_counter()
    nbytes = 0
    for i in range(n):
        s = ds[i % len(ds)]
        nbytes += s["image"].numel() * s["image"].element_size()
    dt = time.perf_counter() - t0
    return n / dt, nbytes / n


def loader_rate(ds, workers, batch, batches):
    import torch

    dl = torch.utils.data.DataLoader(ds, batch_size=batch, shuffle=True, num_workers=workers, drop_last=True,
                                     persistent_workers=False)
    it = iter(dl)
    next(it)  # worker start-up
    t0 = time.perf_counter()
    k = 0
    for _ in range(batches):
        try:
            next(it)
        except StopIteration:
            it = iter(dl)
            next(it)
        k += 1
    return k * batch / (time.perf_counter() - t0)


def shm_loader_rate(ds, workers, batch, batches, device=None, consume=False):
    """The shared-memory batch ring (data/shm_loader.py), consumed like the trainer does: through
    the DevicePrefetcher when a GPU is present (pinned ring -> async H2D), else on the host.
    ``consume``: also build the network input of every batch (device_input.batch_images: the GPU
    jitter if the samples carry it, flip, normalise), as the trainer's step does."""
    from deep_vision_amd.data.device_input import batch_images
    from deep_vision_amd.data.loader import DevicePrefetcher
    from deep_vision_amd.data.shm_loader import ShmBatchLoader

    ld = ShmBatchLoader(ds, batch, num_workers=workers, shuffle=True, drop_last=True, rank=0, world=1)
    try:
        src = DevicePrefetcher(ld, device) if device else ld
        it = iter(src)
        next(it)  # worker start-up
        t0 = time.perf_counter()
        k = 0
        for _ in range(batches):
            try:
                b = next(it)
            except StopIteration:
                it = iter(src)
                b = next(it)
            if consume and device:
                batch_images(b, device)
            k += 1
        if device:
            import torch

            torch.cuda.synchronize()
        return k * batch / (time.perf_counter() - t0), ld.pinned
    finally:
        ld.close()


def gpu_costs(batch, reps=20):
    import torch

    from deep_vision_amd.data.device_input import normalize_u8

    if not torch.cuda.is_available():
        return None
    dev = torch.device("cuda")
    u8 = torch.randint(0, 256, (batch, 224, 224, 3), dtype=torch.uint8).pin_memory()
    f32 = torch.randn(batch, 3, 224, 224).pin_memory()
    flip = torch.randint(0, 2, (batch,), dtype=torch.bool).pin_memory()
    jit = torch.cat([0.8 + 0.4 * torch.rand(batch, 3), torch.stack([torch.randperm(3) for _ in range(batch)]).float()],
                    1).pin_memory()
    res = {}
    for name, fn in (("h2d_fp32_chw", lambda: f32.to(dev, non_blocking=True)),
                     ("h2d_u8_hwc", lambda: u8.to(dev, non_blocking=True)),
                     ("h2d_u8_plus_normalize", lambda: normalize_u8(u8.to(dev, non_blocking=True),
                                                                    flip.to(dev, non_blocking=True))),
                     ("h2d_u8_plus_jitter_normalize", lambda: normalize_u8(u8.to(dev, non_blocking=True),
                                                                           flip.to(dev, non_blocking=True),
                                                                           jitter=jit.to(dev, non_blocking=True)))):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        res[name + "_ms"] = round((time.perf_counter() - t0) / reps * 1e3, 3)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=256)
    ap.add_argument("--per-worker", type=int, default=128, help="samples timed in the single-process rate")
    ap.add_argument("--workers", default="1,2,4,8")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--batches", type=int, default=8)
    ap.add_argument("--gpu-batch", type=int, default=256)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from deep_vision_amd.data import transforms as T
    from deep_vision_amd.data.datasets import ImageNet2012Dataset

    rec = {"images": a.images, "cpu_count": os.cpu_count()}
    with tempfile.TemporaryDirectory() as d:
        imgdir = os.path.join(d, "train_flatten")
        os.makedirs(imgdir)
        t0 = time.perf_counter()
        syn = make_jpegs(imgdir, a.images)
        rec["jpeg_gen_s"] = round(time.perf_counter() - t0, 2)
        arms = {"reference_fp32": ImageNet2012Dataset(imgdir, syn, T.imagenet_train_transform(device_normalize=False)),
                "device_normalize_u8": ImageNet2012Dataset(imgdir, syn, T.imagenet_train_transform(device_normalize=True),
                                                           decode_min_side=256),
                "device_normalize_u8_zero_copy_decode": ImageNet2012Dataset(
                    imgdir, syn, T.imagenet_train_transform(device_normalize=True), decode_min_side=256,
                    zero_copy=True),
                # ColorJitter draws in the worker, the pixels jittered on the GPU (transforms.JitterDraw)
                "device_normalize_u8_device_jitter": ImageNet2012Dataset(
                    imgdir, syn, T.imagenet_train_transform(device_normalize=True, device_jitter=True),
                    decode_min_side=256)}
        for name, ds in arms.items():
            r, b = per_worker_rate(ds, a.per_worker)
            rec[name] = {"per_worker_img_s": round(r, 1), "bytes_per_img": int(b), "loader_img_s": {}}
            for w in [int(v) for v in a.workers.split(",") if v]:
                if w <= (os.cpu_count() or 1):
                    rec[name]["loader_img_s"][w] = round(loader_rate(ds, w, a.batch, a.batches), 1)
            if name in ("device_normalize_u8", "device_normalize_u8_device_jitter"):
                import torch

                dev = "cuda" if torch.cuda.is_available() else None
                rec[name]["shm_loader_img_s"] = {}
                for w in [int(v) for v in a.workers.split(",") if v]:
                    r, pinned = shm_loader_rate(ds, w, a.batch, a.batches, dev)
                    rec[name]["shm_loader_img_s"][w] = round(r, 1)
                    rec[name]["shm_ring_pinned"] = pinned
            print(name, json.dumps(rec[name]), flush=True)
    rec["h2d_bytes_ratio_fp32_over_u8"] = round(rec["reference_fp32"]["bytes_per_img"] /
                                                rec["device_normalize_u8"]["bytes_per_img"], 2)
    g = gpu_costs(a.gpu_batch)
    if g:
        rec["gpu_batch"] = a.gpu_batch
        rec.update(g)
    print(json.dumps(rec), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
