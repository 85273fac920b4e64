"""End-to-end ImageNet-trainer run on generated JPEGs (no dataset download): the reference's
entry point ``ResNet/pytorch/train.py -m <model>`` over a flattened ImageNet-like directory of
~500x375 JPEGs (bench/input_pipeline.py make_jpegs, 10 synsets) -- decode + resize-crop in the
loader workers, the shared-memory batch ring, GPU jitter / flip / normalise, the native training
step, validation and the per-epoch checkpoint. Prints the trainer log and its timer summary
(``--profile timer``: samples/s over the epoch's wall clock, input wait included).

python tools/e2e_imagenet.py [--model resnet50] [--images 6144] [--batch 128] [--workers 16]
                             [--epochs 2] [--device cuda]
"""
import argparse
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bench"))
from input_pipeline import make_jpegs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--images", type=int, default=6144)
    ap.add_argument("--val-images", type=int, default=512)
    ap.add_argument("--unique", type=int, default=2048,
                    help="distinct JPEGs generated; the rest of --images are hard links to them (same decode work)")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--workers", type=int, default=16)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--device", default=None)
    ap.add_argument("--extra", default="", help="more trainer arguments")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as d:
        tr, va = os.path.join(d, "train_flatten"), os.path.join(d, "val_flatten")
        os.makedirs(tr)
        os.makedirs(va)
        t0 = time.perf_counter()
        u = min(a.unique, a.images)
        make_jpegs(tr, u, seed=0)  # writes <d>/synsets.txt
        names = sorted(os.listdir(tr))
        for i in range(u, a.images):  # nXXXXXXXX_<i>.JPEG: the synset prefix keeps the label
            src = names[i % u]
            os.link(os.path.join(tr, src), os.path.join(tr, f"{src.split('_')[0]}_{i}.JPEG"))
        make_jpegs(va, a.val_images, seed=1)
        print(f"[e2e] {a.images} train ({u} distinct) + {a.val_images} val JPEGs in {time.perf_counter() - t0:.1f} s",
              flush=True)
        cmd = [sys.executable, os.path.join(ROOT, "ResNet", "pytorch", "train.py"), "-m", a.model, "--data-dir", d,
               "--epochs", str(a.epochs), "--batch-size", str(a.batch), "--workers", str(a.workers),
               "--val-steps", "2", "--profile", "timer", "--checkpoint-dir", os.path.join(d, "ckpt")]
        if a.device:
            cmd += ["--device", a.device]
        cmd += a.extra.split()
        print("[e2e] " + " ".join(cmd[1:]), flush=True)
        t0 = time.perf_counter()
        rc = subprocess.call(cmd, cwd=d)
        print(f"[e2e] trainer exit {rc} after {time.perf_counter() - t0:.1f} s", flush=True)
        sys.exit(rc)


if __name__ == "__main__":
    main()
