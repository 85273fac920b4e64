"""Per-parameter gradient cosine, native bf16 vs torch fp32 (debug aid)."""
import copy
import sys

import torch

sys.path.insert(0, ".")
from deep_vision_amd.ops.common import set_backend  # noqa: E402
from deep_vision_amd import models as M  # noqa: E402
from deep_vision_amd.ops import loss as L  # noqa: E402


def cos(a, b):
    a, b = a.float().flatten(), b.float().flatten()
    return (a @ b / (a.norm() * b.norm()).clamp_min(1e-12)).item()


def run(name, make, x, loss_fn, train):
    torch.manual_seed(0)
    m = make().cuda().train(train)
    r = copy.deepcopy(m)
    out = m(x)
    loss_fn(out).backward()
    set_backend("torch")
    out_r = r(x)
    loss_fn(out_r).backward()
    set_backend("native")
    print(f"== {name} train={train}")
    for (n, pa), pb in zip(m.named_parameters(), r.parameters()):
        if pb.grad is None:
            continue
        c = cos(pa.grad, pb.grad)
        print(f"  {n:50s} cos={c:.4f} |a|={pa.grad.norm():.3e} |b|={pb.grad.norm():.3e}")


x = torch.randn(2, 3, 128, 128, device="cuda")
t = torch.rand(2, 16, 32, 32, device="cuda") * (torch.rand(2, 16, 32, 32, device="cuda") > 0.9)
for train in (False, True):
    run("hourglass", lambda: M.StackedHourglassNetwork(num_stack=2), x, lambda ys: sum(L.heatmap_mse(y, t) for y in ys), train)
