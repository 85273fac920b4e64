"""Shared-memory loader vs stock DataLoader on the box's CPUs (bench/input_pipeline.py's JPEGs and
transforms), both host-only and the shm ring through the device prefetcher; per worker count."""
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from input_pipeline import loader_rate, make_jpegs, shm_loader_rate  # noqa: E402


def main():
    import torch

    from deep_vision_amd.data import transforms as T
    from deep_vision_amd.data.datasets import ImageNet2012Dataset

    workers = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "4,8,16").split(",")]
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    out = {"batch": batch}
    with tempfile.TemporaryDirectory() as d:
        imgdir = os.path.join(d, "train_flatten")
        os.makedirs(imgdir)
        syn = make_jpegs(imgdir, 1536)
        ds = ImageNet2012Dataset(imgdir, syn, T.imagenet_train_transform(device_normalize=True), decode_min_side=256)
        # the trainer's default: ColorJitter draws in the worker, the pixels jittered on the GPU
        dsj = ImageNet2012Dataset(imgdir, syn, T.imagenet_train_transform(device_normalize=True, device_jitter=True),
                                  decode_min_side=256)
        dev = "cuda" if torch.cuda.is_available() else None
        for w in workers:
            r = {"stock": round(loader_rate(ds, w, batch, 24), 1)}
            r["shm_host"] = round(shm_loader_rate(ds, w, batch, 24, None)[0], 1)
            if dev:
                r["shm_device"] = round(shm_loader_rate(ds, w, batch, 24, dev, consume=True)[0], 1)
                r["shm_device_gpu_jitter"] = round(shm_loader_rate(dsj, w, batch, 24, dev, consume=True)[0], 1)
            else:
                r["shm_host_gpu_jitter_draws"] = round(shm_loader_rate(dsj, w, batch, 24, None)[0], 1)
            out[w] = r
            print(w, json.dumps(r), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    t0 = time.time()
    main()
