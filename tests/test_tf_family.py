"""TF-family data / checkpoint / observability parity on CPU:

* ImageNet writer -> 15-feature Example (bbox lists from the bbox CSV, human text) -> TF1 reader
  (9-feature parse, legacy-TF bilinear aspect resize, crop / flip, RGB mean subtraction,
  label - 1) -> one ``alexnet2_tf`` Keras-mode training step writing the Keras checkpoint /
  pickled-loggers names and TensorBoard scalars;
* TensorBoard event files: our writer round-trips, and our reader parses the reference's own
  checked-in Keras event file (R/LeNet/tensorflow/tensorboard/...).
"""
import glob
import os
import pickle

import numpy as np
import pytest
import torch

REF = "/root/reference"
SYN = ["n01440764", "n01443537", "n01484850", "n01491361"]


def _jpeg(path, h, w, seed):
    from PIL import Image

    rng = np.random.default_rng(seed)
    Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)).save(path, quality=90)


def _imagenet_shards(tmp_path):
    from deep_vision_amd.data.builders import build_imagenet

    flat = tmp_path / "flat"
    flat.mkdir()
    for i in range(16):
        _jpeg(flat / f"{SYN[i % 4]}_{i}.JPEG", 40 + 3 * i, 64 - i, i)
    (tmp_path / "synsets.txt").write_text("".join(f"{s} x\n" for s in SYN))
    (tmp_path / "meta.txt").write_text("".join(f"{s}\tclass {s}\n" for s in SYN))
    (tmp_path / "boxes.csv").write_text("n01440764_0.JPEG,0.1000,0.2000,0.5000,0.6000\n"
                                        "n01440764_0.JPEG,0.0000,0.0000,1.0000,1.0000\n"
                                        "n01443537_1.JPEG,0.2500,0.2500,0.7500,0.7500\n")
    root = tmp_path / "dataset" / "tfrecord"
    for split, shards in (("tfrecord_train", 2), ("tfrecord_val", 1)):
        build_imagenet(str(flat), str(tmp_path / "synsets.txt"), str(root / split), split="train" if shards == 2 else
                       "validation", num_shards=shards, workers=1, bbox_csv=str(tmp_path / "boxes.csv"),
                       metadata_file=str(tmp_path / "meta.txt"))
    return tmp_path / "dataset"


def test_imagenet_writer_reader_roundtrip(tmp_path):
    from deep_vision_amd.data.imagenet_tf import CHANNEL_MEANS, ImageNetTFRecordDataset
    from deep_vision_amd.data.tfrecord import decode_example, example_values

    data = _imagenet_shards(tmp_path)
    tr = ImageNetTFRecordDataset(str(data / "tfrecord" / "tfrecord_train" / "*"), True)
    va = ImageNetTFRecordDataset(str(data / "tfrecord" / "tfrecord_val" / "*"), False)
    assert len(tr) == len(va) == 16
    seen = {}
    for i in range(len(va)):
        ex = decode_example(va.index[i])
        fname = example_values(ex, "image/filename")[0].decode()
        syn = example_values(ex, "image/class/synset")[0].decode()
        label = example_values(ex, "image/class/label")[0]
        assert label == SYN.index(syn) + 1  # builder: 1-based (TF-models)
        assert example_values(ex, "image/class/text")[0].decode() == f"class {syn}"
        xmin = example_values(ex, "image/object/bbox/xmin", [])
        blab = example_values(ex, "image/object/bbox/label", [])
        if fname == "n01440764_0.JPEG":
            assert np.allclose(xmin, [0.1, 0.0]) and list(blab) == [label, label]
            assert np.allclose(example_values(ex, "image/object/bbox/ymax"), [0.6, 1.0])
        elif fname == "n01443537_1.JPEG":
            assert np.allclose(xmin, [0.25])
        else:
            assert len(xmin) == 0
        item = va[i]
        assert item["annotation"] == label - 1  # reader: 0-based
        assert item["image"].shape == (3, 224, 224) and item["image"].dtype == torch.float32
        seen[fname] = item
    # mean subtraction: a uint8 image minus the RGB means stays within [-mean, 255 - mean]
    img = seen["n01440764_0.JPEG"]["image"]
    for c, m in enumerate(CHANNEL_MEANS):
        assert img[c].min() >= -m - 1e-3 and img[c].max() <= 255 - m + 1e-3
    # training items: random crop + flip of the same resized image -> same shape, 0-based label
    assert tr[3]["image"].shape == (3, 224, 224) and 0 <= tr[3]["annotation"] < 4


def test_tf1_legacy_bilinear_resize():
    """TF1 resize_bilinear(align_corners=False): src = dst * in/out, no half-pixel offset."""
    from deep_vision_amd.data.imagenet_tf import smallest_size_at_least, tf1_resize_bilinear

    img = np.array([[0.0, 10.0], [20.0, 30.0]], dtype=np.float32)[:, :, None]
    out = tf1_resize_bilinear(img, 4, 4)[:, :, 0]
    # rows sample 0, 0.5, 1, 1.5 (clamped neighbour) of the input
    assert np.allclose(out[0], [0, 5, 10, 10]) and np.allclose(out[:, 0], [0, 10, 20, 20])
    assert np.allclose(out[1, 1], 15.0)
    assert smallest_size_at_least(375, 500) == (256, 341)  # truncating int32 casts
    assert smallest_size_at_least(500, 333) == (384, 256)


def test_keras_mode_step_writes_reference_layout(tmp_path):
    """alexnet2_tf: TFRecord input -> 1 training step -> ``alexnet2-tf-{ts}-checkpoint-epoch-1.pt``,
    ``alexnet2-tf-{ts}-loggers-epoch-1.pkl`` (7 series incl. lr, R/ResNet/tensorflow/train.py:
    81-144) and TensorBoard epoch scalars under ``{tb}/alexnet2-tf-{ts}``."""
    from deep_vision_amd.config import get_config
    from deep_vision_amd.train.classification import resolve_checkpoint, run_epochs
    from deep_vision_amd.utils.tensorboard import read_scalars

    data = _imagenet_shards(tmp_path)
    ck = tmp_path / "ck"
    last, loggers = run_epochs(get_config("alexnet2_tf"), None, device="cpu", data_dir=str(data), epochs=1,
                               max_steps=1, val_steps=1, batch_size=8, num_workers=0, checkpoint_dir=str(ck) + "/",
                               tensorboard_dir=str(tmp_path / "tb"))
    name = os.path.basename(last)
    assert name.startswith("alexnet2-tf-") and name.endswith("-checkpoint-epoch-1.pt")
    stem = name[: -len("-checkpoint-epoch-1.pt")]
    pk = ck / f"{stem}-loggers-epoch-1.pkl"
    with open(pk, "rb") as f:  # written by our own trainer
        lg = pickle.load(f)
    assert sorted(lg) == sorted(["train_loss", "train_top1_acc", "train_top5_acc", "val_loss", "val_top1_acc",
                                 "val_top5_acc", "lr"])
    assert lg["lr"]["value"] == [0.01] and lg["val_loss"]["epochs"] == [1]
    assert 0.0 <= lg["val_top1_acc"]["value"][0] <= 1.0
    ev = glob.glob(str(tmp_path / "tb" / stem / "events.out.tfevents.*"))
    assert len(ev) == 1
    sc = read_scalars(ev[0])
    assert {"loss", "acc", "val_loss", "val_acc", "lr"} <= set(sc)
    assert sc["lr"][0][:2] == (0, pytest.approx(0.01))
    st = torch.load(last, map_location="cpu", weights_only=True)
    assert st["epoch"] == 1 and {"model", "optimizer", "scheduler", "loggers"} <= set(st)
    assert resolve_checkpoint("latest", get_config("alexnet2_tf"), str(ck)) == last


def test_tensorboard_writer_roundtrip(tmp_path):
    from deep_vision_amd.utils.tensorboard import SummaryWriter, read_scalars

    with SummaryWriter(str(tmp_path)) as w:
        for s in range(5):
            w.add_scalar("train/loss", 1.0 / (s + 1), s)
        w.add_scalars({"a": 2.5, "b": -1.0}, 7)
    files = glob.glob(str(tmp_path / "events.out.tfevents.*"))
    assert len(files) == 1
    sc = read_scalars(files[0])
    assert [v[0] for v in sc["train/loss"]] == list(range(5))
    assert sc["train/loss"][2][1] == pytest.approx(1 / 3, rel=1e-6)
    assert sc["a"][0][:2] == (7, 2.5) and sc["b"][0][:2] == (7, -1.0)


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "LeNet/tensorflow/tensorboard")),
                    reason="reference tree not mounted")
def test_tensorboard_reader_parses_reference_keras_file():
    """The reference's Keras TensorBoard file (LeNet-5 TF, 50 epochs): our reader recovers the
    four per-epoch series; the last val_acc equals the README's final 98.22 %."""
    from deep_vision_amd.utils.tensorboard import read_scalars

    f = glob.glob(os.path.join(REF, "LeNet/tensorflow/tensorboard/*/events.out.tfevents.*"))[0]
    sc = read_scalars(f)
    assert set(sc) == {"loss", "acc", "val_loss", "val_acc"}
    assert all(len(v) == 50 for v in sc.values())
    assert [s for s, _, _ in sc["val_acc"]] == list(range(50))
    assert sc["val_acc"][-1][1] == pytest.approx(0.9822, abs=1e-4)
