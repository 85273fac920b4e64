"""YOLOv3 detection: decode + NMS (Postprocessor(iou .5, score .5)) -- the demo_mscoco.ipynb flow
(R/YOLO/tensorflow/demo_mscoco.ipynb cells 3-10) as a script.

usage: python inference.py -c ./models/model-v1.0.1-epoch-56-loss-42.0143.pt images...
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from deep_vision_amd.inference import main  # noqa: E402

if __name__ == "__main__":
    main(["detect"] + sys.argv[1:])
