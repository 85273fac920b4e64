"""ImageNet -> TFRecord shards (R/Datasets/ILSVRC2012/build_imagenet_tfrecord.py: 1024 train /
128 val shards, labels 1..1000). TF-free: deep_vision_amd.data.builders (process pool).

usage: python build_imagenet_tfrecord.py --flat-dir ../dataset/train_flatten --synsets synsets.txt \
           --out ../dataset/tfrecords [--split train|validation] [--shards 1024]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from deep_vision_amd.data.builders import main  # noqa: E402

if __name__ == "__main__":
    main(["imagenet"] + sys.argv[1:])
