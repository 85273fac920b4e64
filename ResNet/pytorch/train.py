"""ResNet / VGG / Inception / AlexNet / MobileNet PT trainer: `python train.py -m <model> [-c <ckpt>]`
(R/ResNet/pytorch/train.py:541-562). One process per GPU: add `--nproc 8`."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from deep_vision_amd.train.classification import main  # noqa: E402

CHOICES = ["alexnet1", "alexnet2", "vgg16", "vgg19", "inception1", "resnet34", "resnet50", "resnet152", "mobilenet1",
           "shufflenet1"]

if __name__ == "__main__":
    main(choices=CHOICES)
