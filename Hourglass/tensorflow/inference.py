"""Stacked Hourglass keypoints (argmax + quarter-pixel shift), the demo_hourglass_pose.ipynb flow
(R/Hourglass/tensorflow/demo_hourglass_pose.ipynb cells 2-8) as a script.

usage: python inference.py -c ./models/model-v1.0.1-epoch-50-loss-1.0654.pt images...
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from deep_vision_amd.inference import main  # noqa: E402

if __name__ == "__main__":
    main(["pose"] + sys.argv[1:])
