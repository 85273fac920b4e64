"""Module-by-module native-vs-torch comparison of a model forward (debug aid): forward hooks
record every submodule output in both backends; prints the cosine similarity per module."""
import copy
import sys

import torch

sys.path.insert(0, ".")
from deep_vision_amd.ops.common import set_backend  # noqa: E402
from deep_vision_amd import models as M  # noqa: E402


def cos(a, b):
    a, b = a.float().flatten(), b.float().flatten()
    return (a @ b / (a.norm() * b.norm()).clamp_min(1e-12)).item()


def record(model):
    out = {}

    def mk(name):
        def hook(mod, inp, o):
            if isinstance(o, torch.Tensor):
                out[name] = o.detach()
            elif isinstance(o, (list, tuple)) and o and isinstance(o[0], torch.Tensor):
                out[name] = o[0].detach()
        return hook

    for n, m in model.named_modules():
        if n:
            m.register_forward_hook(mk(n))
    return out


def compare(name, make, x, limit=60, min_cos=0.999):
    torch.manual_seed(0)
    m = make().cuda().train()
    r = copy.deepcopy(m)
    a, b = record(m), record(r)
    m(x)
    set_backend("torch")
    r(x)
    set_backend("native")
    shown = 0
    for k in a:
        if k in b and a[k].shape == b[k].shape:
            c = cos(a[k], b[k])
            if c < min_cos and shown < limit:
                print(f"{name} {k:50s} {tuple(a[k].shape)} cos={c:.5f}", flush=True)
                shown += 1
    print(f"{name}: done ({len(a)} modules)", flush=True)


which = sys.argv[1:] or ["hourglass", "yolo", "centernet"]
if "hourglass" in which:
    compare("hourglass", lambda: M.StackedHourglassNetwork(num_stack=2), torch.randn(2, 3, 128, 128, device="cuda"))
if "yolo" in which:
    compare("yolo", lambda: M.YoloV3(80), torch.randn(2, 3, 128, 128, device="cuda"))
if "centernet" in which:
    compare("centernet", lambda: M.ObjectsAsPoints(num_classes=8), torch.randn(2, 3, 128, 128, device="cuda"))
