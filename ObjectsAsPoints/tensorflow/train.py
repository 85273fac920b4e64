"""CenterNet (Objects as Points) trainer (R/ObjectsAsPoints/tensorflow/train.py, which never ran:
this one trains with the paper's focal + L1 objective)."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from deep_vision_amd.train.detection import main  # noqa: E402

if __name__ == "__main__":
    main("centernet")
