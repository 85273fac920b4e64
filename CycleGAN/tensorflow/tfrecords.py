"""CycleGAN image folders -> trainA/trainB/testA/testB TFRecords (R/CycleGAN/tensorflow/tfrecords.py:9-70).

usage: python tfrecords.py --dataset monet2photo [--datasets-dir datasets] [--out tfrecords]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from deep_vision_amd.data.builders import main  # noqa: E402

if __name__ == "__main__":
    main(["cyclegan"] + sys.argv[1:])
