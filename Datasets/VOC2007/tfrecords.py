"""VOC 2007 -> TFRecord shards (R/Datasets/VOC2007/tfrecords.py: XML parse, the COCO Example schema).

usage: python tfrecords.py --root VOCdevkit/VOC2007 --names voc_2007_names.txt --out ../../dataset/tfrecords_voc
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from deep_vision_amd.data.builders import main  # noqa: E402

if __name__ == "__main__":
    main(["voc"] + sys.argv[1:])
