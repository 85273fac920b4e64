"""Keras-origin LeNet trainer, re-expressed on deep_vision_amd (PyTorch-ROCm + native gfx950 kernels).
Keys map to the Keras variants of the models (Keras BN / padding semantics), see
deep_vision_amd/config.py (R/LeNet/tensorflow/train.py)."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from deep_vision_amd.train.classification import main  # noqa: E402

ALIASES = {"resnet50": "resnet50_tf", "resnet152": "resnet152_tf", "alexnet2": "alexnet2_tf", "lenet5": "lenet5_tf",
           "mobilenetv1_1.0": "mobilenet1_tf"}

if __name__ == "__main__":
    argv = sys.argv[1:]
    for i, a in enumerate(argv):
        if i and argv[i - 1] in ("-m", "--model") and a in ALIASES:
            argv[i] = ALIASES[a]
    main(argv, choices=['lenet5_tf'], default="lenet5_tf")
