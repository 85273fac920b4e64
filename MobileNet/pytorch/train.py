"""MobileNet PT trainer: `python train.py -m <model> [-c <ckpt>]` (same CLI as R/MobileNet/pytorch/train.py)."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from deep_vision_amd.train.classification import main  # noqa: E402

if __name__ == "__main__":
    main(choices=['mobilenet1'], default="mobilenet1")
