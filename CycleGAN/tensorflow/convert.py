"""Export the generator (R/CycleGAN/tensorflow/convert.py:7-13 converts a SavedModel to TFLite;
here: safetensors weights + a TorchScript trace, the portable PyTorch deployment formats).

usage: python convert.py -c ./checkpoints-monet2photo/ckpt-N.pt --out ./generator [--size 256]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from deep_vision_amd.inference import main  # noqa: E402

if __name__ == "__main__":
    main(["export", "-m", "cyclegan_generator"] + sys.argv[1:])
