"""Run-to-run gradient agreement of identical fwd+bwd passes (default model ResNet-50, batch 8,
96x96): two default-mode (atomic) runs and one deterministic-mode run from the same weights, per
parameter cosine of A vs B (atomic noise) and A vs det, worst first. Used to bisect nondeterminism
and to check that the deterministic mode computes the same gradients.

    python tools/diag_noise.py [model] [batch] [size]
"""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_vision_amd import models as M  # noqa: E402
from deep_vision_amd import ops as F  # noqa: E402


def grads(base, x, y, det):
    from deep_vision_amd import set_deterministic

    set_deterministic(det)
    try:
        torch.manual_seed(5)
        m = copy.deepcopy(base)
        loss = F.cross_entropy(m(x), y)
        loss.backward()
        torch.cuda.synchronize()
        return loss.item(), [(n, p.grad.detach().float().flatten().clone()) for n, p in m.named_parameters()]
    finally:
        set_deterministic(False)


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    bs = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    size = int(sys.argv[3]) if len(sys.argv) > 3 else 96
    torch.manual_seed(0)
    base = M.get_model(name).cuda()
    x = torch.randn(bs, 3, size, size, device="cuda")
    y = torch.randint(0, 1000, (bs,), device="cuda")
    la, ga = grads(base, x, y, False)
    lb, gb = grads(base, x, y, False)
    lc, gc = grads(base, x, y, True)
    # sensitivity baseline: the default mode on an input perturbed at the 1e-6 level
    xp = x * (1 + 1e-6 * torch.randn_like(x))
    ld, gd = grads(base, xp, y, False)
    cos = torch.nn.functional.cosine_similarity
    rows = []
    for (n, a), (_, b), (_, c) in zip(ga, gb, gc):
        rows.append((cos(a, c, dim=0).item(), cos(a, b, dim=0).item(), n, a.norm().item(), c.norm().item()))
    print(f"perturbed-input run: loss {ld!r}, total cos A-perturbed "
          f"{cos(torch.cat([t for _, t in ga]), torch.cat([t for _, t in gd]), dim=0).item():.6f}")
    cat = lambda g: torch.cat([t for _, t in g])  # noqa: E731
    print(f"{name} batch {bs} @{size}: losses A {la!r} B {lb!r} det {lc!r}")
    print(f"total cos A-B {cos(cat(ga), cat(gb), dim=0).item():.6f}  A-det {cos(cat(ga), cat(gc), dim=0).item():.6f}")
    print("worst A-det (cos A-det, cos A-B, name, |A|, |det|):")
    for r in sorted(rows)[:12]:
        print(f"   {r[0]:.6f} {r[1]:.6f} {r[2]} {r[3]:.4g} {r[4]:.4g}")


if __name__ == "__main__":
    main()
