"""First layer whose forward output differs between two deep copies of one model (same input):
forward hooks capture every leaf module's output in both runs."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_vision_amd import models as M  # noqa: E402
from deep_vision_amd import ops as F  # noqa: E402


def capture(m, x, y, backward):
    outs = []

    def hook(mod, inp, out, name=None):
        if isinstance(out, torch.Tensor):
            outs.append((name, out.detach().float().clone()))

    hs = [mod.register_forward_hook(lambda mod, i, o, n=n: hook(mod, i, o, n)) for n, mod in m.named_modules() if n]
    loss = F.cross_entropy(m(x), y)
    if backward:
        loss.backward()
    torch.cuda.synchronize()
    for h in hs:
        h.remove()
    return outs, loss.item()


def main():
    torch.manual_seed(0)
    base = M.get_model("resnet50").cuda()
    x = torch.randn(8, 3, 96, 96, device="cuda")
    y = torch.randint(0, 1000, (8,), device="cuda")
    for backward in (False, False, True, True, True):
        ra, la = capture(copy.deepcopy(base), x, y, backward)
        rb, lb = capture(copy.deepcopy(base), x, y, backward)
        print(f"backward={backward} losses {la!r} {lb!r}  captured {len(ra)} outputs")
        shown = 0
        for (n, a), (_, b) in zip(ra, rb):
            d = (a - b).abs().max().item()
            if d > 0 and shown < 4:
                print(f"   differs at {n}: max|a-b| {d:.4g} (max|a| {a.abs().max().item():.4g}) "
                      f"frac {((a != b).float().mean().item()):.3g}")
                shown += 1


if __name__ == "__main__":
    main()
