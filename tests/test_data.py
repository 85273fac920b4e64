"""Input pipeline and offline tooling on CPU: TFRecord / Example wire compatibility (checked
against protobuf's own parser with the tf.train.Example schema built at runtime), IDX files
(incl. the reference's checked-in MNIST label files), transforms, dataset builders -> readers
round trips, native batch normalisation, inference / export CLI."""
import io
import json
import os

import numpy as np
import pytest
import torch

from deep_vision_amd.data import tfrecord as T

REF = "/root/reference"


def _example_classes():
    """tf.train.Example message classes built from a runtime FileDescriptorProto."""
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    fd = descriptor_pb2.FileDescriptorProto(name="dv_example.proto", package="tensorflow", syntax="proto3")
    F = descriptor_pb2.FieldDescriptorProto

    def msg(name, fields, nested=()):
        m = fd.message_type.add(name=name)
        for fname, num, typ, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=typ, label=label)
            if tname:
                f.type_name = tname
        for n in nested:
            m.nested_type.append(n)
        return m

    msg("BytesList", [("value", 1, F.TYPE_BYTES, F.LABEL_REPEATED, None)])
    msg("FloatList", [("value", 1, F.TYPE_FLOAT, F.LABEL_REPEATED, None)])
    msg("Int64List", [("value", 1, F.TYPE_INT64, F.LABEL_REPEATED, None)])
    feat = msg("Feature", [("bytes_list", 1, F.TYPE_MESSAGE, F.LABEL_OPTIONAL, ".tensorflow.BytesList"),
                           ("float_list", 2, F.TYPE_MESSAGE, F.LABEL_OPTIONAL, ".tensorflow.FloatList"),
                           ("int64_list", 3, F.TYPE_MESSAGE, F.LABEL_OPTIONAL, ".tensorflow.Int64List")])
    od = feat.oneof_decl.add(name="kind")
    for f in feat.field:
        f.oneof_index = 0
    entry = descriptor_pb2.DescriptorProto(name="FeatureEntry")
    entry.field.add(name="key", number=1, type=F.TYPE_STRING, label=F.LABEL_OPTIONAL)
    entry.field.add(name="value", number=2, type=F.TYPE_MESSAGE, label=F.LABEL_OPTIONAL, type_name=".tensorflow.Feature")
    entry.options.map_entry = True
    msg("Features", [("feature", 1, F.TYPE_MESSAGE, F.LABEL_REPEATED, ".tensorflow.Features.FeatureEntry")], [entry])
    msg("Example", [("features", 1, F.TYPE_MESSAGE, F.LABEL_OPTIONAL, ".tensorflow.Features")])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    get = message_factory.GetMessageClass
    return get(pool.FindMessageTypeByName("tensorflow.Example")), od


def test_example_wire_compatible_with_protobuf():
    Example, _ = _example_classes()
    feats = {"image/encoded": T.bytes_feature(b"\x00\xff jpeg"), "image/object/bbox/xmin": T.float_list_feature([0.25, 0.5]),
             "image/object/class/label": T.int64_list_feature([3, 79, -1]), "image/height": T.int64_feature(416)}
    raw = T.encode_example(feats)
    ex = Example()
    ex.ParseFromString(raw)
    f = ex.features.feature
    assert f["image/encoded"].bytes_list.value[0] == b"\x00\xff jpeg"
    assert list(f["image/object/bbox/xmin"].float_list.value) == [0.25, 0.5]
    assert list(f["image/object/class/label"].int64_list.value) == [3, 79, -1]
    # protobuf-serialised (packed, map order of its choosing) -> native decoder
    back = T.decode_example(ex.SerializeToString())
    assert back["image/object/class/label"] == ("int64", [3, 79, -1])
    assert back["image/height"] == ("int64", [416])
    assert back["image/object/bbox/xmin"][1] == pytest.approx([0.25, 0.5])


def test_tfrecord_framing_and_index(tmp_path):
    p = str(tmp_path / "x.tfrecord")
    recs = [os.urandom(n) for n in (0, 1, 7, 1000)]
    with T.TFRecordWriter(p) as w:
        for r in recs:
            w.write(r)
    assert list(T.tfrecord_iterator(p)) == recs
    idx = T.TFRecordIndex([p])
    assert [idx[i] for i in range(len(idx))] == recs
    assert T.native().crc32c(b"123456789") == 0xE3069283  # CRC-32C check value
    data = bytearray(open(p, "rb").read())
    data[20] ^= 0xFF  # corrupt a payload byte
    open(p, "wb").write(bytes(data))
    with pytest.raises(RuntimeError, match="crc"):
        list(T.tfrecord_iterator(p))


def test_idx_and_reference_mnist_labels(tmp_path):
    from deep_vision_amd.data.datasets import MnistDataset, read_idx, write_idx

    a = np.random.default_rng(0).integers(0, 255, (5, 28, 28)).astype(np.uint8)
    write_idx(str(tmp_path / "im"), a)
    assert np.array_equal(read_idx(str(tmp_path / "im")), a)
    lab = os.path.join(REF, "Datasets/MNIST/t10k-labels-idx1-ubyte")
    if not os.path.exists(lab):
        pytest.skip("reference tree not mounted")
    y = read_idx(lab)
    assert y.shape == (10000,) and y.max() == 9 and list(y[:5]) == [7, 2, 1, 0, 4]
    ds = MnistDataset(None, lab, synthetic_images=True)
    s = ds[0]
    assert s["image"].shape == (1, 32, 32) and int(s["label"]) == 7


def test_reference_synsets():
    from deep_vision_amd.data.datasets import read_synsets

    p = os.path.join(REF, "Datasets/ILSVRC2012/synsets.txt")
    if not os.path.exists(p):
        pytest.skip("reference tree not mounted")
    l2i, i2n = read_synsets(p)
    assert len(l2i) == 1000 and l2i["n01440764"] == 0


def test_transforms_and_native_normalize():
    from deep_vision_amd.data import transforms as TR

    img = (np.random.default_rng(0).random((300, 400, 3)) * 255).astype(np.uint8)
    s = TR.imagenet_train_transform()({"image": img, "annotation": 3})
    assert s["image"].shape == (3, 224, 224) and s["annotation"] == 3
    s = TR.Rescale(256)({"image": img, "annotation": 0})
    assert s["image"].shape[:2] == (256, 341)
    src = (np.random.default_rng(1).random((2, 5, 6, 3)) * 255).astype(np.uint8)
    dst = np.empty((2, 3, 5, 6), np.float32)
    T.native().normalize_batch(src, dst, [0.485, 0.456, 0.406], [0.229, 0.224, 0.225], 255.0, 3)
    ref = (src.transpose(0, 3, 1, 2) / 255.0 - np.array([0.485, 0.456, 0.406]).reshape(1, 3, 1, 1)) / \
        np.array([0.229, 0.224, 0.225]).reshape(1, 3, 1, 1)
    assert np.allclose(dst, ref, atol=1e-5)


def _jpeg(path, w, h, seed):
    from PIL import Image

    a = (np.random.default_rng(seed).random((h, w, 3)) * 255).astype(np.uint8)
    Image.fromarray(a).save(path, format="JPEG")


def test_coco_builder_to_yolo_dataset(tmp_path):
    from deep_vision_amd.data import builders as B
    from deep_vision_amd.data.yolo import YoloTFRecordDataset

    imgs = tmp_path / "img"
    imgs.mkdir()
    for i in range(3):
        _jpeg(str(imgs / f"{i}.jpg"), 64 + 8 * i, 48, i)
    ann = {"images": [{"id": i, "file_name": f"{i}.jpg"} for i in range(3)],
           "categories": [{"id": 1, "name": "person"}, {"id": 3, "name": "car"}],
           "annotations": [{"image_id": i, "category_id": 3 if i else 1, "bbox": [4, 4, 20, 16]} for i in range(3)]}
    json.dump(ann, open(tmp_path / "ann.json", "w"))
    res = B.build_coco(str(tmp_path / "ann.json"), str(imgs), str(tmp_path / "rec"), "train", num_shards=2, workers=1)
    assert sum(n for _, n in res) == 3
    files = sorted(str(tmp_path / "rec" / f) for f in os.listdir(tmp_path / "rec"))
    assert os.path.basename(files[0]) == "train-00000-of-00002"
    ds = YoloTFRecordDataset(files, False, num_classes=2, output_shape=(64, 64))
    img, (s, m, l) = ds[0]
    assert img.shape == (3, 64, 64) and -1 <= img.min() and img.max() <= 1
    assert s.shape == (8, 8, 3, 7) and (s[..., 4].sum() + m[..., 4].sum() + l[..., 4].sum()) == 1


def test_mpii_and_cyclegan_builders(tmp_path):
    from deep_vision_amd.data import builders as B
    from deep_vision_amd.data.pose import MPIITFRecordDataset

    _jpeg(str(tmp_path / "p.jpg"), 120, 100, 3)
    joints = [[30 + 3 * k, 20 + 4 * k] for k in range(16)]
    joints[5] = [-1, -1]
    anno = [{"image": "p.jpg", "joints": joints, "joints_visibility": [1] * 16, "center": [60, 50], "scale": 0.3}]
    json.dump(anno, open(tmp_path / "mpii.json", "w"))
    B.build_mpii(str(tmp_path / "mpii.json"), str(tmp_path), str(tmp_path / "mp"), num_shards=1, workers=1)
    ds = MPIITFRecordDataset([str(tmp_path / "mp" / "train-00000-of-00001")], False)
    img, hm = ds[0]
    assert img.shape == (3, 256, 256) and hm.shape == (16, 64, 64) and hm.max() == pytest.approx(12.0)
    d = tmp_path / "datasets" / "toy" / "trainA"
    d.mkdir(parents=True)
    _jpeg(str(d / "a.jpg"), 32, 32, 1)
    (d / "broken.jpg").write_bytes(b"not a jpeg")
    out = B.build_cyclegan(str(tmp_path / "datasets"), "toy", str(tmp_path / "tf"))
    assert out["trainA"] == 1 and out["trainB"] == 0


def test_inference_classify_and_export(tmp_path):
    from deep_vision_amd import inference as I
    from deep_vision_amd import models as M

    _jpeg(str(tmp_path / "c.jpg"), 80, 60, 5)
    m = M.get_model("resnet34")
    torch.save({"epoch": 1, "model": {"module." + k: v for k, v in m.state_dict().items()}}, tmp_path / "r.pt")
    r = I.classify("resnet34", str(tmp_path / "r.pt"), [str(tmp_path / "c.jpg")], device="cpu")
    assert len(r[0]) == 5 and sum(p for _, _, p in r[0]) <= 1.0 + 1e-5
    st, ts = I.export("lenet5", None, str(tmp_path / "lenet"), (1, 1, 32, 32))
    assert os.path.getsize(st) > 0 and torch.jit.load(ts)(torch.randn(1, 1, 32, 32)).shape == (1, 10)


def test_imagenet_bbox_xml_to_csv(tmp_path):
    """ImageNet bounding-box XML -> normalised, clipped, ordered CSV (process_bounding_boxes, T1b)."""
    from deep_vision_amd.data.builders import parse_bbox_xml, process_bounding_boxes

    d = tmp_path / "n01440764"
    d.mkdir()
    (d / "n01440764_10.xml").write_text(
        "<annotation><filename>n01440764_10</filename><size><width>200</width><height>100</height></size>"
        "<object><name>n01440764</name><bndbox><xmin>20</xmin><ymin>10</ymin><xmax>220</xmax><ymax>50</ymax></bndbox></object>"
        "<object><name>n09999999</name><bndbox><xmin>0</xmin><ymin>0</ymin><xmax>10</xmax><ymax>10</ymax></bndbox></object>"
        "</annotation>")
    (d / "broken.xml").write_text("<annotation><filename>")
    fname, boxes = parse_bbox_xml(str(d / "n01440764_10.xml"))
    assert fname == "n01440764_10" and len(boxes) == 2
    assert boxes[0][:4] == (0.1, 0.1, 1.0, 0.5)  # xmax 220/200 clipped to 1
    syn = tmp_path / "synsets.txt"
    syn.write_text("n01440764 tench\n")
    out = tmp_path / "boxes.csv"
    n_files, n_boxes, skipped = process_bounding_boxes(str(tmp_path), str(out), str(syn))
    assert (n_files, n_boxes, skipped) == (1, 1, 1)
    assert out.read_text().strip() == "n01440764_10.JPEG,0.1000,0.1000,1.0000,0.5000"


def test_celeba_split_and_val_flatten(tmp_path):
    from deep_vision_amd.data.builders import celeba_split, flatten_imagenet_val

    img = tmp_path / "img"
    img.mkdir()
    for f in ("000001.jpg", "000002.jpg", "000003.jpg"):
        (img / f).write_bytes(b"x")
    attr = tmp_path / "list_attr_celeba.txt"
    attr.write_text("3\nBald Male Young\n000001.jpg -1 1 1\n000002.jpg -1 -1 1\n000003.jpg 1 1 -1\n")
    counts = celeba_split(str(attr), str(img), str(tmp_path / "celeba"))
    assert counts == {"trainA": 2, "trainB": 1}
    assert sorted(os.listdir(tmp_path / "celeba" / "trainA")) == ["000001.jpg", "000003.jpg"]
    val = tmp_path / "val"
    val.mkdir()
    for i in (2, 1):
        (val / f"ILSVRC2012_val_0000000{i}.JPEG").write_bytes(b"y")
    labels = tmp_path / "labels.txt"
    labels.write_text("n01751748\nn09193705\n")
    assert flatten_imagenet_val(str(val), str(labels), str(tmp_path / "vf")) == 2
    assert sorted(os.listdir(tmp_path / "vf")) == ["n01751748_ILSVRC2012_val_00000001.JPEG",
                                                   "n09193705_ILSVRC2012_val_00000002.JPEG"]


def test_uint8_pipeline_matches_float_pipeline():
    """workers ship uint8 HWC crops + a flip draw; flip / ToTensor / Normalize
    on the device (here the CPU arm of data.device_input) equal the reference float pipeline."""
    import random as pyrandom

    import numpy as np

    from deep_vision_amd.data import transforms as T
    from deep_vision_amd.data.device_input import normalize_u8

    rng = np.random.RandomState(0)
    img = rng.randint(0, 256, (300, 420, 3), dtype=np.uint8)
    ref_t = T.Compose([T.Rescale(256), T.CenterCrop(224), T.ToTensor(), T.Normalize(T.IMAGENET_MEAN, T.IMAGENET_STD)])
    u8_t = T.Compose([T.Rescale(256), T.CenterCrop(224), T.ToUint8(flip_p=1.0)])
    ref = ref_t({"image": img, "annotation": 3})["image"]
    s = u8_t({"image": img, "annotation": 3})
    assert s["image"].dtype == torch.uint8 and tuple(s["image"].shape) == (224, 224, 3) and s["flip"]
    assert s["image"].numel() * s["image"].element_size() * 4 == ref.numel() * ref.element_size()  # 4x fewer bytes
    batch = torch.utils.data.default_collate([s, {**s, "flip": False}])
    out = normalize_u8(batch["image"], batch["flip"])
    assert torch.allclose(out[0], ref.flip(2), atol=1e-4)
    assert torch.allclose(out[1], ref, atol=1e-4)
    pyrandom.seed(0)
    tr = T.imagenet_train_transform(device_normalize=True)({"image": img, "annotation": 1})
    assert tr["image"].dtype == torch.uint8 and isinstance(tr["flip"], bool)


def test_device_jitter_draws_and_bytes_match_worker_jitter():
    """transforms.JitterDraw + data.device_input.jitter_u8 (the pixels jittered after the batch
    leaves the worker) give the same RNG draws, the same flip draw and the same bytes as the
    worker-side FastColorJitter, for every order of the three enhancers."""
    import random as pyrandom

    import numpy as np

    from deep_vision_amd.data import transforms as T
    from deep_vision_amd.data.device_input import jitter_u8, normalize_u8

    rng = np.random.RandomState(1)
    imgs = [rng.randint(0, 256, (300 + 7 * k, 420 - 5 * k, 3), dtype=np.uint8) for k in range(6)]
    host, dev = [], []
    for k, img in enumerate(imgs):
        pyrandom.seed(100 + k)
        np.random.seed(100 + k)
        host.append(T.imagenet_train_transform(device_normalize=True)({"image": img.copy(), "annotation": 0}))
        pyrandom.seed(100 + k)
        np.random.seed(100 + k)
        dev.append(T.imagenet_train_transform(device_normalize=True, device_jitter=True)({"image": img.copy(),
                                                                                          "annotation": 0}))
    orders = {tuple(int(v) for v in d["jitter"][3:]) for d in dev}
    assert len(orders) >= 3  # the seeds cover several enhancer orders
    for h, d in zip(host, dev):
        assert h["flip"] == d["flip"]
        assert d["jitter"].dtype == torch.float32 and tuple(d["jitter"].shape) == (6,)
    hb = torch.utils.data.default_collate(host)
    db = torch.utils.data.default_collate(dev)
    assert not torch.equal(hb["image"], db["image"])  # the device form has not jittered yet
    jitter_u8(db["image"], db["jitter"])
    assert torch.equal(hb["image"], db["image"])
    a = normalize_u8(hb["image"], hb["flip"])
    db2 = torch.utils.data.default_collate(dev)
    b = normalize_u8(db2["image"], db2["flip"], jitter=db2["jitter"])
    assert torch.equal(a, b)
