"""Stacked Hourglass trainer, script form (R/Hourglass/tensorflow/train.py:229-240 with its
undefined `epochs` fixed: uses the config's 100)."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from deep_vision_amd.train.detection import main  # noqa: E402

if __name__ == "__main__":
    main("hourglass", tfrecords_default="./dataset/tfrecords_mpii")
