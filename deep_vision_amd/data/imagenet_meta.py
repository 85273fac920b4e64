"""ImageNet-2012 label metadata shipped with the package.

The reference keeps the class list as loose files next to its dataset scripts
(R/Datasets/ILSVRC2012/{synsets.txt, imagenet_2012_metadata.txt, imagenet_2012_synsets.txt,
indices.json, imagenet_2012_validation_synset_labels.txt}); its trainers, notebooks and TFRecord
builder read them from the working directory. Here the same content lives in ONE compressed
table (``meta/imagenet2012.json.gz``: the 1000 synset ids in label order, their human-readable
names, and the 50,000 validation labels as class indices), and every one of those files can be
re-materialised byte for byte (``write_reference_files``) -- ``tests/test_imagenet_meta.py``
pins each against the reference's SHA-256.

Label order is the sorted-synset order: index i = line i of synsets.txt (the PyTorch trainers'
0-based labels); the TFRecord builder and the TF1 reader use i + 1.
"""
from __future__ import annotations

import functools
import gzip
import json
import os

_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "meta", "imagenet2012.json.gz")

# SHA-256 of the reference's files (R/Datasets/ILSVRC2012/*), reproduced by write_reference_files
REFERENCE_SHA256 = {
    "synsets.txt": "b6e5b90376a998304703176bc829997a99fc461ecbb75e855db80b3d5b76d827",
    "imagenet_2012_metadata.txt": "ea92b64bd83ab8335792dec1c6e8028010d440943c7a76e0fb1ab986f941c62e",
    "imagenet_2012_synsets.txt": "385e0240499426c022b773be1ae4da780f057b89c9694c7f47199f62746b6edd",
    "indices.json": "6fc259c92562c13483975ae536d840c6ca7229fb73409f35512a8ae052b0bbbd",
    "imagenet_2012_validation_synset_labels.txt": "2707a43f27dcd55fef87fbef0730966cb91c3aba99eb0c9e6f021217a553a3b1",
}


@functools.lru_cache(maxsize=1)
def _table():
    with gzip.open(_PATH, "rt", encoding="utf-8") as f:
        return json.load(f)


def wnids() -> list:
    """The 1000 synset ids (``n01440764`` ...) in label order."""
    return list(_table()["wnids"])


def names() -> list:
    """Human-readable class names in label order (``'tench, Tinca tinca'`` ...)."""
    return list(_table()["names"])


def label_to_idx() -> dict:
    return {w: i for i, w in enumerate(_table()["wnids"])}


def idx_to_name() -> dict:
    """idx -> name, the content of the notebooks' indices.json."""
    return dict(enumerate(_table()["names"]))


def val_labels() -> list:
    """Class index of each of the 50,000 validation images (ILSVRC2012_val_00000001 first)."""
    return list(_table()["val_labels"])


def render(name: str) -> str:
    """Text of one reference metadata file, byte-identical to the reference copy."""
    t = _table()
    w, n = t["wnids"], t["names"]
    if name == "synsets.txt":
        return "\n".join(f"{a} {b}" for a, b in zip(w, n))
    if name == "imagenet_2012_metadata.txt":
        return "\n".join(f"{a}\t{b}" for a, b in zip(w, n))
    if name == "imagenet_2012_synsets.txt":
        return "\n".join(w)
    if name == "indices.json":
        return json.dumps({str(i): b for i, b in enumerate(n)}, indent=4)
    if name == "imagenet_2012_validation_synset_labels.txt":
        return "\n".join(w[i] for i in t["val_labels"])
    raise KeyError(name)


def write_reference_files(out_dir: str, files=None) -> list:
    """Write the reference's metadata files into ``out_dir`` (the layout its scripts expect:
    ``../dataset/synsets.txt`` etc.). Returns the written paths."""
    os.makedirs(out_dir, exist_ok=True)
    out = []
    for name in files or REFERENCE_SHA256:
        p = os.path.join(out_dir, name)
        with open(p, "w", encoding="utf-8", newline="") as f:
            f.write(render(name))
        out.append(p)
    return out


def default_synsets_file(cache_dir: str | None = None) -> str:
    """Path of a synsets.txt materialised from the packaged table (for code that wants a file)."""
    d = cache_dir or os.path.join(os.path.expanduser("~"), ".cache", "deep_vision_amd")
    p = os.path.join(d, "synsets.txt")
    if not os.path.isfile(p):
        write_reference_files(d, ["synsets.txt"])
    return p


def main(argv=None):
    import argparse

    ap = argparse.ArgumentParser(description="write the ImageNet-2012 label metadata files")
    ap.add_argument("out_dir")
    a = ap.parse_args(argv)
    for p in write_reference_files(a.out_dir):
        print(p)


if __name__ == "__main__":
    main()
