"""First module whose forward output differs between the default and the deterministic mode
(bisects a deterministic-mode statistics bug): forward hooks record every leaf module's output.

    python tools/diag_det.py [model] [batch] [size]
"""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_vision_amd import models as M  # noqa: E402


def run(base, x, det):
    from deep_vision_amd import set_deterministic

    set_deterministic(det)
    outs = []
    m = copy.deepcopy(base)
    hooks = []
    for n, mod in m.named_modules():
        def hook(mod, inp, out, n=n):
            o = out[0] if isinstance(out, (tuple, list)) else out
            if isinstance(o, torch.Tensor):
                outs.append((n, type(mod).__name__, o.detach().float().clone()))
        hooks.append(mod.register_forward_hook(hook))
    try:
        m(x)
        torch.cuda.synchronize()
    finally:
        set_deterministic(False)
    bns = [(n, b.running_mean.clone(), b.running_var.clone()) for n, b in m.named_modules()
           if isinstance(b, torch.nn.BatchNorm2d)]
    return outs, bns


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    bs = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    size = int(sys.argv[3]) if len(sys.argv) > 3 else 96
    torch.manual_seed(0)
    base = M.get_model(name).cuda()
    x = torch.randn(bs, 3, size, size, device="cuda")
    a, ba = run(base, x, False)
    b, bb = run(base, x, True)
    shown = 0
    for (n, t, u), (_, _, v) in zip(a, b):
        d = ((u - v).norm() / u.norm().clamp_min(1e-12)).item() if u.shape == v.shape else float("nan")
        if d > 1e-3 and shown < 10:
            print(f"output differs: {n} ({t}) rel {d:.4g} shape {tuple(u.shape)}")
            shown += 1
    shown = 0
    for (n, m1, v1), (_, m2, v2) in zip(ba, bb):
        dm = ((m1 - m2).norm() / m1.norm().clamp_min(1e-12)).item()
        dv = ((v1 - v2).norm() / v1.norm().clamp_min(1e-12)).item()
        if (dm > 1e-4 or dv > 1e-4) and shown < 10:
            print(f"running stats differ: {n} mean {dm:.4g} var {dv:.4g}")
            shown += 1
    print("done", len(a), "outputs compared")


if __name__ == "__main__":
    main()
