"""CycleGAN translation A->B / B->A from the latest checkpoint (R/CycleGAN/tensorflow/inference.py:11-72).

usage: python inference.py --checkpoint-dir ./checkpoints-monet2photo [--direction a2b] images...
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from deep_vision_amd.inference import main  # noqa: E402

if __name__ == "__main__":
    main(["translate"] + sys.argv[1:])
