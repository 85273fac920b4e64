"""COCO 2017 -> TFRecord shards (R/Datasets/MSCOCO/tfrecords.py:160-196; 64 train / 8 val shards).

usage: python tfrecords.py --annotations instances_train2017.json --images train2017 --out ../../dataset/tfrecords
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from deep_vision_amd.data.builders import main  # noqa: E402

if __name__ == "__main__":
    main(["coco"] + sys.argv[1:])
