"""Offline dataset tooling: raw datasets -> TFRecord shards, TF-free.

* COCO 2017 (R/Datasets/MSCOCO/tfrecords.py:37-196): annotations grouped by image, boxes
  normalised (and asserted in [0, 1]), class ids remapped to 0..79, 64 / 8 shards
* VOC 2007 / 2012 (R/Datasets/VOC2007/tfrecords.py:124-206): XML parse, same Example schema
* MPII (R/Datasets/MPII/tfrecords_mpii.py): writes the schema the Hourglass *reader* expects --
  int64 parts x/y/v in pixels (-1 = missing), center x/y and scale -- fixing the reference
  writer (float parts through an Int64List, no center/scale)
* ImageNet (R/Datasets/ILSVRC2012/build_imagenet_tfrecord.py): the TF-models schema with
  labels 1..1000 (0 = background); 1024 / 128 shards
* CycleGAN image folders (R/CycleGAN/tensorflow/tfrecords.py:9-70): trainA/B, testA/B
  (unreadable files are skipped instead of crashing, A19)
* ``flatten_imagenet`` / ``flatten_imagenet_val``: the train_flatten / val_flatten layout of
  flatten-script.sh / flatten-val-script.sh (T1c)
* ``process_bounding_boxes``: ImageNet bbox XML -> normalised, clipped CSV (T1b)
* ``celeba_split``: CelebA -> CycleGAN trainA / trainB by attribute (T5)

Shards are written by a process pool (the reference fans out with ray / threads).
"""
from __future__ import annotations

import io
import json
import os
import shutil
import xml.etree.ElementTree as ET
from collections import defaultdict
from multiprocessing import Pool
from typing import Dict, List, Sequence

from .tfrecord import (TFRecordWriter, bytes_feature, bytes_list_feature, encode_example, float_list_feature,
                       int64_feature, int64_list_feature, shard_name)


def read_jpeg(path):
    """Raw JPEG bytes (re-encoded at quality 95 when not an RGB JPEG) and (width, height)."""
    from PIL import Image

    with open(path, "rb") as f:
        content = f.read()
    with Image.open(path) as im:
        width, height = im.size
        if im.format != "JPEG" or im.mode != "RGB":
            with io.BytesIO() as out:
                im.convert("RGB").save(out, format="JPEG", quality=95)
                content = out.getvalue()
    return content, width, height


def detection_example(filepath, annos):
    """annos: [{'class_id', 'class_text', 'xmin', 'ymin', 'xmax', 'ymax'}] in pixels."""
    content, width, height = read_jpeg(filepath)
    xs0, ys0, xs1, ys1 = [], [], [], []
    for a in annos:
        b = (float(a["xmin"]) / width, float(a["ymin"]) / height, float(a["xmax"]) / width, float(a["ymax"]) / height)
        assert all(0 <= v <= 1 for v in b), (filepath, b)
        xs0.append(b[0])
        ys0.append(b[1])
        xs1.append(b[2])
        ys1.append(b[3])
    return encode_example({
        "image/height": int64_feature(height), "image/width": int64_feature(width), "image/depth": int64_feature(3),
        "image/object/bbox/xmin": float_list_feature(xs0), "image/object/bbox/ymin": float_list_feature(ys0),
        "image/object/bbox/xmax": float_list_feature(xs1), "image/object/bbox/ymax": float_list_feature(ys1),
        "image/object/class/label": int64_list_feature([a["class_id"] for a in annos]),
        "image/object/class/text": bytes_list_feature([a["class_text"] for a in annos]),
        "image/encoded": bytes_feature(content), "image/filename": bytes_feature(os.path.basename(filepath)),
    })


def _write_shard(args):
    path, items, fn = args
    n = 0
    with TFRecordWriter(path) as w:
        for it in items:
            rec = fn(*it)
            if rec is not None:
                w.write(rec)
                n += 1
    return path, n


def write_sharded(items: Sequence, fn, out_dir: str, prefix: str, num_shards: int, workers: int = 8):
    """Split ``items`` (argument tuples of ``fn``) into ``num_shards`` files ``prefix-0000k-of-N``."""
    os.makedirs(out_dir, exist_ok=True)
    num_shards = max(1, min(num_shards, len(items))) if items else 1
    jobs = [(os.path.join(out_dir, shard_name(prefix, s, num_shards)), items[s::num_shards], fn)
            for s in range(num_shards)]
    if workers <= 1:
        return [_write_shard(j) for j in jobs]
    with Pool(min(workers, len(jobs))) as p:
        return p.map(_write_shard, jobs)


# ------------------------------------------------------------------ COCO
def coco_items(annotation_file: str, image_dir: str):
    with open(annotation_file) as f:
        d = json.load(f)
    cats = sorted(c["id"] for c in d["categories"])
    cid = {c: i for i, c in enumerate(cats)}  # 91 sparse ids -> 0..79
    names = {c["id"]: c["name"] for c in d["categories"]}
    files = {im["id"]: im["file_name"] for im in d["images"]}
    groups: Dict[int, List[dict]] = defaultdict(list)
    for a in d["annotations"]:
        x, y, w, h = a["bbox"]
        groups[a["image_id"]].append({"class_id": cid[a["category_id"]], "class_text": names[a["category_id"]],
                                      "xmin": x, "ymin": y, "xmax": x + w, "ymax": y + h})
    return [(os.path.join(image_dir, files[i]), g) for i, g in sorted(groups.items())]


def build_coco(annotation_file, image_dir, out_dir, split="train", num_shards=64, workers=8):
    return write_sharded(coco_items(annotation_file, image_dir), detection_example, out_dir, split, num_shards, workers)


# ------------------------------------------------------------------ VOC
def voc_items(voc_root: str, names: Sequence[str], image_set: str = "trainval"):
    names_map = {n: i for i, n in enumerate(names)}
    ids_file = os.path.join(voc_root, "ImageSets", "Main", image_set + ".txt")
    ids = [l.strip() for l in open(ids_file)] if os.path.exists(ids_file) else \
        [f[:-4] for f in sorted(os.listdir(os.path.join(voc_root, "Annotations")))]
    items = []
    for i in ids:
        root = ET.parse(os.path.join(voc_root, "Annotations", i + ".xml")).getroot()
        fn = root.find(".//filename").text
        annos = []
        for obj in root.findall(".//object"):
            bb = obj.find("bndbox")
            name = obj.find("name").text
            annos.append({"class_text": name, "class_id": names_map[name],
                          **{k: int(float(bb.find(k).text)) for k in ("xmin", "ymin", "xmax", "ymax")}})
        items.append((os.path.join(voc_root, "JPEGImages", fn), annos))
    return items


def build_voc(voc_root, names_file, out_dir, image_set="trainval", split="train", num_shards=4, workers=4):
    names = [l.strip() for l in open(names_file) if l.strip()]
    return write_sharded(voc_items(voc_root, names, image_set), detection_example, out_dir, split, num_shards, workers)


# ------------------------------------------------------------------ MPII
def mpii_example(filepath, anno):
    """anno: {'joints': [[x, y], ...16], 'joints_visibility': [...], 'center': [x, y], 'scale': s}."""
    content, width, height = read_jpeg(filepath)
    xs = [int(round(j[0])) if j[0] >= 0 else -1 for j in anno["joints"]]
    ys = [int(round(j[1])) if j[1] >= 0 else -1 for j in anno["joints"]]
    v = [0 if jv == 0 else 2 for jv in anno["joints_visibility"]]
    return encode_example({
        "image/height": int64_feature(height), "image/width": int64_feature(width), "image/depth": int64_feature(3),
        "image/object/parts/x": int64_list_feature(xs), "image/object/parts/y": int64_list_feature(ys),
        "image/object/parts/v": int64_list_feature(v),
        "image/object/center/x": int64_feature(int(round(anno["center"][0]))),
        "image/object/center/y": int64_feature(int(round(anno["center"][1]))),
        "image/object/scale": float_list_feature([float(anno["scale"])]),
        "image/encoded": bytes_feature(content), "image/filename": bytes_feature(os.path.basename(filepath)),
    })


def build_mpii(annotation_json, image_dir, out_dir, split="train", num_shards=16, workers=8):
    with open(annotation_json) as f:
        annos = json.load(f)
    items = [(os.path.join(image_dir, a["image"]), a) for a in annos]
    return write_sharded(items, mpii_example, out_dir, split, num_shards, workers)


# ------------------------------------------------------------------ ImageNet
def imagenet_example(filepath, label, synset, human="", bboxes=()):
    """The reference's 15-feature Example (R/Datasets/ILSVRC2012/build_imagenet_tfrecord.py:
    184-232): image geometry / colorspace, label (1..1000), synset, human text, the image's
    bounding boxes as four parallel float lists + one label per box, format, filename, JPEG."""
    content, width, height = read_jpeg(filepath)
    xmin = [b[0] for b in bboxes]
    ymin = [b[1] for b in bboxes]
    xmax = [b[2] for b in bboxes]
    ymax = [b[3] for b in bboxes]
    return encode_example({
        "image/height": int64_feature(height), "image/width": int64_feature(width),
        "image/colorspace": bytes_feature(b"RGB"), "image/channels": int64_feature(3),
        "image/class/label": int64_feature(label), "image/class/synset": bytes_feature(synset),
        "image/class/text": bytes_feature(human),
        "image/object/bbox/xmin": float_list_feature(xmin), "image/object/bbox/xmax": float_list_feature(xmax),
        "image/object/bbox/ymin": float_list_feature(ymin), "image/object/bbox/ymax": float_list_feature(ymax),
        "image/object/bbox/label": int64_list_feature([label] * len(xmin)),
        "image/format": bytes_feature(b"JPEG"),
        "image/filename": bytes_feature(os.path.basename(filepath)), "image/encoded": bytes_feature(content),
    })


def build_bounding_box_lookup(bbox_csv):
    """``<file>.JPEG,xmin,ymin,xmax,ymax`` lines (process_bounding_boxes output) -> {file: [box]}
    (build_imagenet_tfrecord.py:643-688)."""
    out = {}
    n = 0
    with open(bbox_csv) as f:
        for line in f:
            parts = line.strip().split(",")
            if len(parts) != 5:
                continue
            out.setdefault(parts[0], []).append(tuple(float(v) for v in parts[1:]))
            n += 1
    return out


def build_synset_lookup(metadata_file):
    """``nXXXXXXXX<TAB>human label`` lines (imagenet_metadata.txt) -> {synset: human}."""
    out = {}
    with open(metadata_file) as f:
        for line in f:
            parts = line.rstrip("\n").split("\t")
            if len(parts) == 2:
                out[parts[0]] = parts[1]
    return out


def build_imagenet(flat_dir, synsets_file=None, out_dir=None, split="train", num_shards=1024, workers=8, bbox_csv=None,
                   metadata_file=None):
    """From a flattened directory (``nXXXXXXXX_*.JPEG``); labels start at 1 (TF-models convention,
    ``data.imagenet_tf.ImageNetTFRecordDataset`` subtracts 1). ``bbox_csv`` /
    ``metadata_file`` fill the bounding-box and human-text features by file name / synset."""
    from . import imagenet_meta

    # default: the packaged synset list / human-readable names
    syn = [l.split()[0] for l in open(synsets_file) if l.strip()] if synsets_file else imagenet_meta.wnids()
    idx = {s: i + 1 for i, s in enumerate(syn)}
    boxes = build_bounding_box_lookup(bbox_csv) if bbox_csv else {}
    human = (build_synset_lookup(metadata_file) if metadata_file
             else dict(zip(imagenet_meta.wnids(), imagenet_meta.names())))
    items = []
    for f in sorted(os.listdir(flat_dir)):
        s0 = f.split("_")[0]
        if s0 in idx:
            # the bbox CSV is keyed by the original file name (flattened val files carry a synset prefix)
            key = f if f in boxes else f[len(s0) + 1:]
            items.append((os.path.join(flat_dir, f), idx[s0], s0, human.get(s0, ""), tuple(boxes.get(key, ()))))
    print("Found %d images with bboxes out of %d images" % (sum(1 for it in items if it[4]), len(items)))
    return write_sharded(items, imagenet_example, out_dir, split, num_shards, workers)


def flatten_imagenet(train_dir, out_dir):
    """train/nXXXX/*.JPEG -> out_dir/nXXXX_*.JPEG (hard links when possible)."""
    os.makedirs(out_dir, exist_ok=True)
    n = 0
    for syn in sorted(os.listdir(train_dir)):
        d = os.path.join(train_dir, syn)
        if not os.path.isdir(d):
            continue
        for f in os.listdir(d):
            dst = os.path.join(out_dir, f if f.startswith(syn + "_") else f"{syn}_{f}")
            try:
                os.link(os.path.join(d, f), dst)
            except OSError:
                shutil.copy(os.path.join(d, f), dst)
            n += 1
    return n


def flatten_imagenet_val(val_dir, labels_file, out_dir):
    """val/ILSVRC2012_val_*.JPEG + one synset per line (imagenet_2012_validation_synset_labels.txt,
    in file-name order) -> out_dir/nXXXX_ILSVRC2012_val_*.JPEG (flatten-val-script.sh, T1c)."""
    labels = [l.strip() for l in open(labels_file) if l.strip()]
    files = sorted(f for f in os.listdir(val_dir) if f.upper().endswith((".JPEG", ".JPG")))
    if len(files) != len(labels):
        raise ValueError(f"{len(files)} validation images but {len(labels)} labels")
    os.makedirs(out_dir, exist_ok=True)
    for f, syn in zip(files, labels):
        dst = os.path.join(out_dir, f"{syn}_{f}")
        try:
            os.link(os.path.join(val_dir, f), dst)
        except OSError:
            shutil.copy(os.path.join(val_dir, f), dst)
    return len(files)


def parse_bbox_xml(path, synsets=None):
    """One ImageNet bounding-box XML (R/Datasets/ILSVRC2012/process_bounding_boxes.py:119-169):
    every box normalised by the image size, clipped to [0, 1], min/max ordered. Returns
    (filename, [(xmin, ymin, xmax, ymax, synset)]) or None when the file does not parse."""
    try:
        root = ET.parse(path).getroot()
    except ET.ParseError:
        return None
    fname = root.findtext("filename") or os.path.splitext(os.path.basename(path))[0]
    size = root.find("size")
    width = float(size.findtext("width")) if size is not None else 0.0
    height = float(size.findtext("height")) if size is not None else 0.0
    boxes = []
    for obj in root.iter("object"):
        syn = obj.findtext("name") or ""
        if synsets is not None and syn not in synsets:
            continue
        bb = obj.find("bndbox")
        if bb is None or width <= 0 or height <= 0:
            continue
        x0, y0 = float(bb.findtext("xmin")) / width, float(bb.findtext("ymin")) / height
        x1, y1 = float(bb.findtext("xmax")) / width, float(bb.findtext("ymax")) / height
        x0, x1 = sorted((min(max(x0, 0.0), 1.0), min(max(x1, 0.0), 1.0)))
        y0, y1 = sorted((min(max(y0, 0.0), 1.0), min(max(y1, 0.0), 1.0)))
        boxes.append((x0, y0, x1, y1, syn))
    return fname, boxes


def process_bounding_boxes(xml_dir, out_csv, synsets_file=None):
    """Directory tree of bbox XMLs -> CSV lines ``<image>.JPEG,xmin,ymin,xmax,ymax`` (the
    reference's output format; the TFRecord builder looks boxes up by file name)."""
    synsets = set(l.split()[0] for l in open(synsets_file) if l.strip()) if synsets_file else None
    n_files = n_boxes = skipped = 0
    with open(out_csv, "w") as out:
        for dirpath, _, files in sorted(os.walk(xml_dir)):
            for f in sorted(files):
                if not f.endswith(".xml"):
                    continue
                r = parse_bbox_xml(os.path.join(dirpath, f), synsets)
                if r is None:
                    skipped += 1
                    continue
                fname, boxes = r
                if not fname.upper().endswith(".JPEG"):
                    fname += ".JPEG"
                for x0, y0, x1, y1, _ in boxes:
                    out.write(f"{fname},{x0:.4f},{y0:.4f},{x1:.4f},{y1:.4f}\n")
                    n_boxes += 1
                n_files += 1
    return n_files, n_boxes, skipped


def celeba_split(attr_file, image_dir, out_root, attribute="Male"):
    """CelebA -> CycleGAN folders by one binary attribute (R/CycleGAN/tensorflow/celeba.py:1-24:
    Male -> trainA, the rest -> trainB). ``list_attr_celeba.txt`` format: count line, header
    line of attribute names, then ``<file> <+1|-1> ...``."""
    lines = [l.split() for l in open(attr_file) if l.strip()]
    header = lines[1]
    col = header.index(attribute)
    counts = {"trainA": 0, "trainB": 0}
    for d in counts:
        os.makedirs(os.path.join(out_root, d), exist_ok=True)
    for row in lines[2:]:
        f, vals = row[0], row[1:]
        dst = "trainA" if int(vals[col]) > 0 else "trainB"
        src = os.path.join(image_dir, f)
        if not os.path.exists(src):
            continue
        try:
            os.link(src, os.path.join(out_root, dst, f))
        except OSError:
            shutil.copy(src, os.path.join(out_root, dst, f))
        counts[dst] += 1
    return counts


# ------------------------------------------------------------------ CycleGAN
def image_example(path):
    try:
        content, width, height = read_jpeg(path)
    except Exception as e:  # skip unreadable files (the reference returns None and then crashes)
        print(f"skipping {path}: {e}")
        return None
    return encode_example({"image/encoded": bytes_feature(content), "image/format": bytes_feature(b"JPEG"),
                           "image/width": int64_feature(width), "image/height": int64_feature(height),
                           "image/filename": bytes_feature(os.path.basename(path))})


def build_cyclegan(datasets_dir, name, out_dir="tfrecords"):
    out = {}
    for split in ("trainA", "trainB", "testA", "testB"):
        d = os.path.join(datasets_dir, name, split)
        files = sorted(os.path.join(d, f) for f in os.listdir(d)) if os.path.isdir(d) else []
        path = os.path.join(out_dir, name, f"{split}.tfrecord")
        out[split] = _write_shard((path, [(f,) for f in files], image_example))[1]
        print("Finished converting TFRecords for {}".format(split))
    return out


def main(argv=None):
    import argparse

    ap = argparse.ArgumentParser(description="Build TFRecord shards")
    sub = ap.add_subparsers(dest="cmd", required=True)
    c = sub.add_parser("coco")
    c.add_argument("--annotations", required=True)
    c.add_argument("--images", required=True)
    c.add_argument("--out", default="./dataset/tfrecords")
    c.add_argument("--split", default="train")
    c.add_argument("--shards", type=int, default=64)
    v = sub.add_parser("voc")
    v.add_argument("--root", required=True)
    v.add_argument("--names", required=True)
    v.add_argument("--out", default="./dataset/tfrecords_voc")
    v.add_argument("--image-set", default="trainval")
    v.add_argument("--split", default="train")
    v.add_argument("--shards", type=int, default=4)
    m = sub.add_parser("mpii")
    m.add_argument("--annotations", required=True)
    m.add_argument("--images", required=True)
    m.add_argument("--out", default="./dataset/tfrecords_mpii")
    m.add_argument("--split", default="train")
    m.add_argument("--shards", type=int, default=16)
    i = sub.add_parser("imagenet")
    i.add_argument("--flat-dir", required=True)
    i.add_argument("--synsets", default=None, help="synsets.txt (default: the packaged ImageNet-2012 list)")
    i.add_argument("--out", required=True)
    i.add_argument("--split", default="train")
    i.add_argument("--shards", type=int, default=1024)
    i.add_argument("--bounding-box-file", default=None, help="CSV from the 'bboxes' command")
    i.add_argument("--imagenet-metadata-file", default=None, help="synset<TAB>human label per line")
    g = sub.add_parser("cyclegan")
    g.add_argument("--dataset", required=True)
    g.add_argument("--datasets-dir", default="datasets")
    g.add_argument("--out", default="tfrecords")
    f = sub.add_parser("flatten")
    f.add_argument("--train-dir")
    f.add_argument("--val-dir")
    f.add_argument("--val-labels", help="imagenet_2012_validation_synset_labels.txt")
    f.add_argument("--out", required=True)
    b = sub.add_parser("bboxes")
    b.add_argument("--xml-dir", required=True)
    b.add_argument("--out", required=True)
    b.add_argument("--synsets")
    e = sub.add_parser("celeba")
    e.add_argument("--attr", required=True)
    e.add_argument("--images", required=True)
    e.add_argument("--out", default="datasets/celeba")
    e.add_argument("--attribute", default="Male")
    a = ap.parse_args(argv)
    if a.cmd == "flatten":
        if a.train_dir:
            print("flattened", flatten_imagenet(a.train_dir, a.out), "training images")
        if a.val_dir:
            print("flattened", flatten_imagenet_val(a.val_dir, a.val_labels, a.out), "validation images")
        return
    if a.cmd == "bboxes":
        print("files %d boxes %d skipped %d" % process_bounding_boxes(a.xml_dir, a.out, a.synsets))
        return
    if a.cmd == "celeba":
        print(celeba_split(a.attr, a.images, a.out, a.attribute))
        return
    if a.cmd == "coco":
        build_coco(a.annotations, a.images, a.out, a.split, a.shards)
    elif a.cmd == "voc":
        build_voc(a.root, a.names, a.out, a.image_set, a.split, a.shards)
    elif a.cmd == "mpii":
        build_mpii(a.annotations, a.images, a.out, a.split, a.shards)
    elif a.cmd == "imagenet":
        build_imagenet(a.flat_dir, a.synsets, a.out, a.split, a.shards, bbox_csv=a.bounding_box_file,
                       metadata_file=a.imagenet_metadata_file)
    else:
        build_cyclegan(a.datasets_dir, a.dataset, a.out)


if __name__ == "__main__":
    main()
