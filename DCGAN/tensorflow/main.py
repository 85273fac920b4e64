"""DCGAN on MNIST (R/DCGAN/tensorflow/main.py)."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from deep_vision_amd.train.gan import dcgan_main  # noqa: E402

if __name__ == "__main__":
    dcgan_main()
