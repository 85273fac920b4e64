"""Time one fwd / bwd / optimizer step of a model on the GPU, phase by phase (debug aid).
usage: python tools/debug_step.py <model> [batch] [size]"""
import sys
import time

import torch

sys.path.insert(0, ".")
from deep_vision_amd import models as M  # noqa: E402
from deep_vision_amd import ops as F  # noqa: E402
from deep_vision_amd.train.optim import FusedSGD  # noqa: E402

name = sys.argv[1]
bs = int(sys.argv[2]) if len(sys.argv) > 2 else 8
size = int(sys.argv[3]) if len(sys.argv) > 3 else 224
m = M.get_model(name).cuda().train()
opt = FusedSGD(m.parameters(), lr=0.01, momentum=0.9)
x = torch.randn(bs, 3, size, size, device="cuda")
y = torch.randint(0, 1000, (bs,), device="cuda")


def t(label, fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    print(f"{label:10s} {1e3 * (time.perf_counter() - t0):9.2f} ms", flush=True)
    return r


for it in range(3):
    out = t("fwd", lambda: m(x))
    outs = out if isinstance(out, tuple) else (out,)
    loss = t("loss", lambda: sum(F.cross_entropy(o, y) for o in outs))
    opt.zero_grad()
    t("bwd", lambda: loss.backward())
    t("opt", lambda: opt.step())
    print("loss", loss.item(), flush=True)
