"""Flattened ImageNet directories used by the PT loaders (R/Datasets/ILSVRC2012/flatten-script.sh,
flatten-val-script.sh): train/nXXXX/*.JPEG -> train_flatten/nXXXX_*.JPEG and
val/*.JPEG + synset labels -> val_flatten/nXXXX_ILSVRC2012_val_*.JPEG (hard links).

usage: python flatten.py --train-dir train --out ../dataset/train_flatten
       python flatten.py --val-dir val --val-labels imagenet_2012_validation_synset_labels.txt --out ../dataset/val_flatten
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from deep_vision_amd.data.builders import main  # noqa: E402

if __name__ == "__main__":
    main(["flatten"] + sys.argv[1:])
