"""ImageNet bounding-box XML -> CSV (R/Datasets/ILSVRC2012/process_bounding_boxes.py:171-264).

usage: python process_bounding_boxes.py --xml-dir bboxes/ --out imagenet_2012_bounding_boxes.csv [--synsets synsets.txt]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from deep_vision_amd.data.builders import main  # noqa: E402

if __name__ == "__main__":
    main(["bboxes"] + sys.argv[1:])
