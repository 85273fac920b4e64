"""Long-horizon convergence: native step vs PyTorch autocast-bf16 from one initialisation, on a
streaming learnable synthetic task (reference oracle: the full training logs
R/ResNet/pytorch/logs/resnet34-yanjiali-010319.log, settings R/ResNet/pytorch/train.py:166-184:
SGD lr .1, momentum .9, weight decay 1e-4).

Task: ``classes`` smooth class templates (3x12x12 Gaussian fields upsampled to 224x224); every
training image is a fresh draw ``a * template[c] + noise * N(0,1)``, rolled by a random shift
of up to +-``shift`` pixels and flipped with p=.5. Each step sees a new batch (a function of the
seed and the step index only, so both arms see the same data), so the curve measures learning,
not memorisation of one batch. Every ``every`` steps both arms are evaluated in eval mode (BN
running statistics) on a fixed held-out set.

usage: python tools/convergence.py [--model resnet50] [--batch 256] [--steps 1000] [--seeds 0 1]
                                   [--out profiles/convergence_resnet50.json]
"""
from __future__ import annotations

import argparse
import copy
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_vision_amd import models as M  # noqa: E402
from deep_vision_amd import ops as F  # noqa: E402
from deep_vision_amd.ops.common import set_backend  # noqa: E402
from deep_vision_amd.train.optim import FusedSGD  # noqa: E402


class Task:
    def __init__(self, seed=0, classes=100, size=224, amp=0.6, noise=1.0, shift=24, device="cuda"):
        g = torch.Generator(device="cpu").manual_seed(10_000 + seed)
        t = torch.randn(classes, 3, 12, 12, generator=g)
        t = torch.nn.functional.interpolate(t, size=(size, size), mode="bicubic", align_corners=False)
        self.templ = (t / t.flatten(1).std(1).view(-1, 1, 1, 1)).to(device)
        self.labels = torch.randperm(1000, generator=g)[:classes].to(device)
        self.classes, self.amp, self.noise, self.shift, self.seed = classes, amp, noise, shift, seed
        self.device = device

    def batch(self, bs, index):
        g = torch.Generator(device=self.device).manual_seed(self.seed * 1_000_003 + index)
        cls = torch.randint(0, self.classes, (bs,), device=self.device, generator=g)
        x = self.amp * self.templ[cls]
        sh = torch.randint(-self.shift, self.shift + 1, (2,), device="cpu",
                           generator=torch.Generator().manual_seed(self.seed * 7919 + index)).tolist()
        x = torch.roll(x, shifts=(sh[0], sh[1]), dims=(2, 3))
        flip = torch.rand(bs, device=self.device, generator=g) < 0.5
        x = torch.where(flip.view(-1, 1, 1, 1), x.flip(3), x)
        x = x + self.noise * torch.randn(x.shape, device=self.device, generator=g)
        return x.contiguous(), self.labels[cls]


def _loss(arm, out, y):
    if isinstance(out, tuple):
        out = out[0]
    if arm == "native":
        return F.cross_entropy(out, y), out
    return torch.nn.functional.cross_entropy(out.float(), y), out


def _evaluate(arm, m, task, n_eval, bs):
    m.eval()
    tot, correct, n = 0.0, 0, 0
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16, enabled=arm == "torch-bf16"):
        for i in range(0, n_eval, bs):
            x, y = task.batch(min(bs, n_eval - i), 10_000_000 + i)
            loss, out = _loss(arm, m(x), y)
            k = y.numel()
            tot += loss.item() * k
            correct += (out.float().argmax(1) == y).sum().item()
            n += k
    m.train()
    return tot / n, correct / n


def run(model="resnet50", bs=256, steps=1000, lr=0.1, seed=0, every=100, n_eval=1024, arms=("native", "torch-bf16"),
        log=print, deterministic=False, **task_kw):
    from deep_vision_amd import set_deterministic

    torch.manual_seed(seed)
    base = M.get_model(model).cuda()
    task = Task(seed=seed, **task_kw)
    res = {}
    for arm in arms:
        m = copy.deepcopy(base)
        opt = FusedSGD(m.parameters(), lr=lr, momentum=0.9, weight_decay=1e-4)
        set_backend("native" if arm == "native" else "torch")
        set_deterministic(deterministic and arm == "native")
        losses, evals = [], []
        t0 = time.time()
        try:
            for s in range(steps):
                x, y = task.batch(bs, s)
                opt.zero_grad()
                with torch.autocast("cuda", dtype=torch.bfloat16, enabled=arm == "torch-bf16"):
                    loss, _ = _loss(arm, m(x), y)
                loss.backward()
                opt.step()
                losses.append(loss.detach())
                if (s + 1) % every == 0:
                    el, ea = _evaluate(arm, m, task, n_eval, bs)
                    window = torch.stack(losses[-every:]).float().mean().item()
                    evals.append({"step": s + 1, "train_loss": round(window, 4), "eval_loss": round(el, 4),
                                  "eval_acc": round(ea, 4)})
                    log(f"seed {seed} {arm:10s} step {s + 1:5d} train {window:.4f} eval {el:.4f} acc {ea:.3f} "
                        f"({time.time() - t0:.0f}s)")
        finally:
            set_backend("native")
            set_deterministic(False)
        res[arm] = {"loss": [round(v, 4) for v in torch.stack(losses).float().tolist()], "checkpoints": evals}
    return res


def compare(res):
    """Per-checkpoint differences native - torch-bf16."""
    out = []
    for a, b in zip(res["native"]["checkpoints"], res["torch-bf16"]["checkpoints"]):
        out.append({"step": a["step"], "d_train_loss": round(a["train_loss"] - b["train_loss"], 4),
                    "d_eval_loss": round(a["eval_loss"] - b["eval_loss"], 4),
                    "d_eval_acc": round(a["eval_acc"] - b["eval_acc"], 4)})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--seeds", type=int, nargs="+", default=[0, 1])
    ap.add_argument("--every", type=int, default=100)
    ap.add_argument("--classes", type=int, default=100)
    ap.add_argument("--amp", type=float, default=0.6)
    ap.add_argument("--noise", type=float, default=1.0)
    ap.add_argument("--shift", type=int, default=24)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    out = {"model": a.model, "batch": a.batch, "steps": a.steps, "lr": a.lr, "momentum": 0.9, "weight_decay": 1e-4,
           "task": {"classes": a.classes, "amp": a.amp, "noise": a.noise, "shift": a.shift}, "seeds": {}}
    for seed in a.seeds:
        r = run(a.model, a.batch, a.steps, a.lr, seed, a.every, classes=a.classes, amp=a.amp, noise=a.noise,
                shift=a.shift, log=lambda s: print(s, flush=True))
        out["seeds"][str(seed)] = {"curves": r, "diff": compare(r)}
        for d in out["seeds"][str(seed)]["diff"]:
            print(f"seed {seed} step {d['step']:5d} native-torch: train {d['d_train_loss']:+.4f} "
                  f"eval {d['d_eval_loss']:+.4f} acc {d['d_eval_acc']:+.3f}", flush=True)
        assert all(math.isfinite(v) for v in r["native"]["loss"])
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f)


if __name__ == "__main__":
    main()
