"""MPII -> TFRecord shards in the schema the Hourglass reader expects (fixes
R/Datasets/MPII/tfrecords_mpii.py:54-77).

usage: python tfrecords_mpii.py --annotations mpii_annotations.json --images images --out ../../dataset/tfrecords_mpii
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from deep_vision_amd.data.builders import main  # noqa: E402

if __name__ == "__main__":
    main(["mpii"] + sys.argv[1:])
