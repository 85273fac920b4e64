"""Run-to-run gradient agreement of two identical ResNet-50 fwd+bwd passes (batch 8, 96x96):
per-parameter cosine of the two runs, worst first. Used to bisect nondeterminism."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_vision_amd import models as M  # noqa: E402
from deep_vision_amd import ops as F  # noqa: E402


def run(det=False):
    from deep_vision_amd import set_deterministic

    set_deterministic(det)
    torch.manual_seed(0)
    base = M.get_model(sys.argv[1] if len(sys.argv) > 1 else "resnet50").cuda()
    x = torch.randn(8, 3, 96, 96, device="cuda")
    y = torch.randint(0, 1000, (8,), device="cuda")
    gs = []
    losses = []
    for _ in range(2):
        m = copy.deepcopy(base)
        loss = F.cross_entropy(m(x), y)
        losses.append(loss.item())
        loss.backward()
        torch.cuda.synchronize()
        gs.append([(n, p.grad.detach().float().flatten().clone()) for n, p in m.named_parameters()])
    rows = []
    for (n, a), (_, b) in zip(*gs):
        c = torch.nn.functional.cosine_similarity(a, b, dim=0).item()
        rows.append((c, n, a.norm().item(), b.norm().item()))
    allc = torch.nn.functional.cosine_similarity(torch.cat([a for _, a in gs[0]]), torch.cat([b for _, b in gs[1]]), dim=0)
    print(f"det={det} total cos {allc.item():.6f}  losses {losses[0]!r} {losses[1]!r}")
    for c, n, na, nb in sorted(rows)[:8]:
        print(f"   {c:.6f} {n} |a| {na:.4g} |b| {nb:.4g}")
    print("   last layers:", [(n, round(c, 6)) for c, n, _, _ in rows[-4:]])
    set_deterministic(False)


if __name__ == "__main__":
    run(False)
    run(False)
    run(True)
