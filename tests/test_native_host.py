"""Host-code sanitizers: the native input-pipeline core (csrc/host/io_core.h) built
standalone under AddressSanitizer + UndefinedBehaviorSanitizer and under ThreadSanitizer, then
run: TFRecord round trip, Example decoding with a truncation / mutation fuzz pass, threaded
batch normalisation (csrc/host/selftest/io_selftest.cpp). GPU sanitizers are not available on
this pool, so sanitizers cover host code only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "csrc", "host", "selftest", "io_selftest.cpp")


@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_host_io_core_under_sanitizers(tmp_path, san):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    exe = str(tmp_path / "io_selftest")
    flags = ["-fsanitize=" + san, "-fno-omit-frame-pointer"]
    if "undefined" in san:
        flags.append("-fno-sanitize-recover=undefined")
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-msse4.2", "-pthread", *flags, SRC, "-o", exe],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "io_selftest ok" in r.stdout


def test_color_jitter_matches_pil_enhancers():
    """_io.color_jitter: PIL ImageEnhance Brightness / Contrast / Color bit for bit, in order."""
    import numpy as np
    from PIL import Image, ImageEnhance

    from deep_vision_amd import _io

    rng = np.random.RandomState(0)
    img = rng.randint(0, 256, (37, 53, 3)).astype(np.uint8)
    enh = (ImageEnhance.Brightness, ImageEnhance.Contrast, ImageEnhance.Color)
    for order in ([0, 1, 2], [2, 0, 1], [1, 2, 0]):
        f = [0.83, 1.14, 0.91]
        x = img.copy()
        _io.color_jitter(x, f, order)
        ref = Image.fromarray(img)
        for k in order:
            ref = enh[k](ref).enhance(f[k])
        assert np.array_equal(x, np.asarray(ref)), order


def test_resize_crop_bilinear_geometry():
    """_io.resize_crop: cv2 INTER_LINEAR sampling (half-pixel centres, border clamp) of the crop
    window only; equals a float reference within the 11-bit fixed-point rounding."""
    import numpy as np

    from deep_vision_amd import _io

    rng = np.random.RandomState(1)
    H, W = 47, 61
    src = rng.randint(0, 256, (H, W, 3)).astype(np.uint8)
    oh, ow, cy, cx, ch, cw = 34, 44, 5, 7, 24, 30

    def coords(n_out, n_in, start, count):
        s = (np.arange(start, start + count) + 0.5) * n_in / n_out - 0.5
        s = np.clip(s, 0, None)
        a = np.minimum(np.floor(s).astype(int), n_in - 1)
        return a, np.minimum(a + 1, n_in - 1), s - a

    y0, y1, wy = coords(oh, H, cy, ch)
    x0, x1, wx = coords(ow, W, cx, cw)
    f = src.astype(np.float64)
    top = f[y0][:, x0] * (1 - wx)[None, :, None] + f[y0][:, x1] * wx[None, :, None]
    bot = f[y1][:, x0] * (1 - wx)[None, :, None] + f[y1][:, x1] * wx[None, :, None]
    ref = top * (1 - wy)[:, None, None] + bot * wy[:, None, None]
    out = _io.resize_crop(src, oh, ow, cy, cx, ch, cw)
    assert out.shape == (ch, cw, 3) and np.abs(out.astype(np.float64) - ref).max() <= 1.0


def test_rescale_crop_transform_and_draft_decode(tmp_path):
    """RescaleCrop gives RandomCrop-sized outputs from the Rescale geometry; load_rgb(min_side)
    decodes a large JPEG at a reduced DCT scale whose shorter side stays >= min_side."""
    import numpy as np
    from PIL import Image

    from deep_vision_amd.data import transforms as T
    from deep_vision_amd.data.datasets import load_rgb

    yy, xx = np.mgrid[0:300, 0:420].astype(np.float32)
    img = np.stack([(np.sin(xx / 23 + c) * np.cos(yy / 31) * 0.5 + 0.5) * 255 for c in range(3)], -1).astype(np.uint8)
    out = T.RescaleCrop(256, 224)({"image": img})["image"]
    assert out.shape == (224, 224, 3) and out.dtype == np.uint8
    val = T.RescaleCrop(256, 224, random_crop=False)({"image": img})["image"]
    two = T.CenterCrop(224)(T.Rescale(256)({"image": img}))["image"]
    assert val.shape == two.shape and np.abs(val.astype(int) - two.astype(int)).mean() < 1.5
    p = str(tmp_path / "big.jpg")
    Image.fromarray(np.zeros((1100, 1500, 3), np.uint8) + 90).save(p, quality=90)
    small = load_rgb(p, min_side=256)
    assert min(small.shape[:2]) >= 256 and small.shape[0] < 1100
    assert load_rgb(p).shape[:2] == (1100, 1500)


def test_resize_crop_reads_strided_views_and_zero_copy_decode(tmp_path):
    """_io.resize_crop reads an RGBX-strided view (the decoder's buffer, data/datasets.py load_rgb
    zero_copy) in place and a flipped view through a copy, with the contiguous result; the zero-copy
    decode equals the copying one and stays valid after its image is closed."""
    import gc

    import numpy as np
    from PIL import Image

    from deep_vision_amd import _io
    from deep_vision_amd.data.datasets import load_rgb

    rng = np.random.RandomState(2)
    rgbx = rng.randint(0, 256, (41, 57, 4)).astype(np.uint8)
    view = rgbx[:, :, :3]
    for v in (view, view[:, ::-1], view[::-1]):
        a = _io.resize_crop(v, 36, 50, 3, 4, 30, 40)
        assert np.array_equal(a, _io.resize_crop(np.ascontiguousarray(v), 36, 50, 3, 4, 30, 40))
    paths = []
    for i in range(4):
        p = str(tmp_path / f"im{i}.jpg")
        Image.fromarray(rng.randint(0, 256, (300 + i, 420, 3)).astype(np.uint8)).save(p, quality=90)
        paths.append(p)
    views = [load_rgb(p, 128, zero_copy=True) for p in paths]
    gc.collect()
    _ = [np.full((300, 420, 4), 9, np.uint8) for _ in range(20)]  # reuse freed memory, if any was freed
    for v, p in zip(views, paths):
        assert v.shape[2] == 3 and np.array_equal(v, load_rgb(p, 128))
