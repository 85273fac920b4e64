"""Loss trajectory on one fixed synthetic batch (memorisation): native vs torch backend, same init.
usage: python tools/loss_curve.py [model] [batch] [steps] [lr]"""
import copy
import sys

import torch

sys.path.insert(0, ".")
from deep_vision_amd import models as M  # noqa: E402
from deep_vision_amd import ops as F  # noqa: E402
from deep_vision_amd.ops.common import set_backend  # noqa: E402
from deep_vision_amd.train.optim import FusedSGD  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
bs = int(sys.argv[2]) if len(sys.argv) > 2 else 64
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 30
lr = float(sys.argv[4]) if len(sys.argv) > 4 else 0.1
torch.manual_seed(0)
base = M.get_model(name).cuda()
x = torch.randn(bs, 3, 224, 224, device="cuda")
y = torch.randint(0, 1000, (bs,), device="cuda")
for be in ("native", "torch", "torch-bf16"):
    m = copy.deepcopy(base)
    opt = FusedSGD(m.parameters(), lr=lr, momentum=0.9, weight_decay=1e-4)
    set_backend("native" if be == "native" else "torch")
    ls = []
    for s in range(steps):
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=be == "torch-bf16"):
            out = m(x)
            loss = F.cross_entropy(out, y) if be == "native" else torch.nn.functional.cross_entropy(out.float(), y)
        loss.backward()
        opt.step()
        ls.append(round(loss.item(), 3))
    set_backend("native")
    print(f"{be:10s}", ls, flush=True)
