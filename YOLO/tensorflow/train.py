"""YOLOv3 trainer: `python train.py [--checkpoint ./models/model-v1.0.1-epoch-E-loss-L.pt]`
(R/YOLO/tensorflow/train.py:276-313). TFRecords from ./dataset/tfrecords/{train,val}*; --synthetic
for generated data; --nproc N for one process per GPU."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from deep_vision_amd.train.detection import main  # noqa: E402

if __name__ == "__main__":
    main("yolov3")
