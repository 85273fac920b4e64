"""The ImageNet trainer end to end on JPEG files (CPU): tools/e2e_imagenet.py generates a small
flattened ImageNet-like directory and runs the reference's entry point ``ResNet/pytorch/train.py``
on it -- JPEG decode + resize-crop in the loader workers, the shared-memory batch ring, the ColorJitter
draws shipped with the batch and applied by data.device_input, epoch-0 validation, one training
epoch, validation, the per-epoch checkpoint."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_imagenet_trainer_on_jpegs_cpu(tmp_path):
    env = dict(os.environ, OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "e2e_imagenet.py"), "--model", "mobilenet1",
                        "--images", "48", "--unique", "24", "--val-images", "16", "--batch", "8", "--workers", "2",
                        "--epochs", "1", "--device", "cpu"],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "48 train (24 distinct) + 16 val JPEGs" in out
    assert "Epoch: 0, Validation Set Loss" in out and "Epoch: 1, Validation Set Loss" in out
    assert "[dv-profile] epoch 1:" in out and "samples_per_s" in out
