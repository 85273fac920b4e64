"""CelebA gender split into CycleGAN folders: Male -> trainA, Female -> trainB
(R/CycleGAN/tensorflow/celeba.py:1-24).

usage: python celeba.py --attr list_attr_celeba.txt --images img_align_celeba [--out datasets/celeba]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from deep_vision_amd.data.builders import main  # noqa: E402

if __name__ == "__main__":
    main(["celeba"] + sys.argv[1:])
