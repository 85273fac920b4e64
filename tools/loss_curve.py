"""Loss trajectory of one fixed synthetic batch, native vs torch backends from the same init.

usage: python tools/loss_curve.py [model] [batch] [steps] [lr] [task] [out.json]

task "learnable" (default): 16 classes, every image = 0.5 * its class template + 0.3 * noise,
labels drawn from the 1000-way head; a correct training step drives the cross-entropy from
ln(1000) ~ 6.9 towards 0 within ~100 SGD steps at lr <= 0.05 (SURVEY §7.3 phase 2).
task "random": random images and labels (memorisation).
The three arms share the initial weights: "native" (HIP kernels, bf16), "torch" (PyTorch fp32)
and "torch-bf16" (PyTorch under autocast bf16, the precision-matched reference).
"""
import copy
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_vision_amd import models as M  # noqa: E402
from deep_vision_amd import ops as F  # noqa: E402
from deep_vision_amd.ops.common import set_backend  # noqa: E402
from deep_vision_amd.train.optim import FusedSGD  # noqa: E402


def make_batch(bs, task="learnable", size=224, classes=16, seed=0, noise=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    if task == "random":
        x = torch.randn(bs, 3, size, size, generator=g)
        y = torch.randint(0, 1000, (bs,), generator=g)
    else:
        labels = torch.randperm(1000, generator=g)[:classes]
        templ = torch.randn(classes, 3, size, size, generator=g)
        cls = torch.arange(bs) % classes
        x = 0.5 * templ[cls] + noise * torch.randn(bs, 3, size, size, generator=g)
        y = labels[cls]
    return x.cuda(), y.cuda()


def run_curve(name="resnet50", bs=128, steps=100, lr=0.05, task="learnable", arms=("native", "torch-bf16"), seed=0,
              noise=1.0, deterministic=False):
    """deterministic=True runs the native arm under set_deterministic (a reproducible trajectory on
    any box: no float-atomic accumulation order); the torch arms are unaffected."""
    from deep_vision_amd import set_deterministic

    torch.manual_seed(seed)
    base = M.get_model(name).cuda()
    x, y = make_batch(bs, task, noise=noise)
    curves = {}
    for arm in arms:
        m = copy.deepcopy(base)
        opt = FusedSGD(m.parameters(), lr=lr, momentum=0.9, weight_decay=1e-4)
        set_backend("native" if arm == "native" else "torch")
        set_deterministic(deterministic and arm == "native")
        ls = []
        try:
            for _ in range(steps):
                opt.zero_grad()
                with torch.autocast("cuda", dtype=torch.bfloat16, enabled=arm == "torch-bf16"):
                    out = m(x)
                    if isinstance(out, tuple):
                        out = out[0]
                    if arm == "native":
                        loss = F.cross_entropy(out, y)
                    else:
                        loss = torch.nn.functional.cross_entropy(out.float(), y)
                loss.backward()
                opt.step()
                ls.append(round(loss.item(), 4))
        finally:
            set_backend("native")
            set_deterministic(False)
        curves[arm] = ls
    return curves


def main():
    a = sys.argv[1:]
    name = a[0] if len(a) > 0 else "resnet50"
    bs = int(a[1]) if len(a) > 1 else 128
    steps = int(a[2]) if len(a) > 2 else 100
    lr = float(a[3]) if len(a) > 3 else 0.01
    task = a[4] if len(a) > 4 else "learnable"
    curves = run_curve(name, bs, steps, lr, task, arms=("native", "torch", "torch-bf16"), noise=0.3)
    for arm, ls in curves.items():
        print(f"{arm:10s} first {ls[0]:.3f} last {ls[-1]:.4f} min {min(ls):.4f}  {ls[::10]}", flush=True)
    if len(a) > 5:
        with open(a[5], "w") as f:
            json.dump({"model": name, "batch": bs, "steps": steps, "lr": lr, "task": task, "curves": curves}, f)


if __name__ == "__main__":
    main()
