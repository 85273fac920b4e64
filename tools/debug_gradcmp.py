"""Gradient agreement: native bf16 vs torch fp32 vs torch autocast-bf16 (is a disagreement a bug
or the model's own sensitivity to bf16 rounding?). usage: python tools/debug_gradcmp.py <model> [bs] [size]"""
import copy
import sys

import torch

sys.path.insert(0, ".")
from deep_vision_amd import models as M  # noqa: E402
from deep_vision_amd import ops as F  # noqa: E402
from deep_vision_amd.ops.common import set_backend  # noqa: E402


def cos(a, b):
    a, b = a.float().flatten(), b.float().flatten()
    return (a @ b / (a.norm() * b.norm()).clamp_min(1e-20)).item()


name = sys.argv[1]
bs = int(sys.argv[2]) if len(sys.argv) > 2 else 4
size = int(sys.argv[3]) if len(sys.argv) > 3 else 224
torch.manual_seed(0)
x = torch.randn(bs, 3, size, size, device="cuda")
y = torch.randint(0, 1000, (bs,), device="cuda")
base = M.get_model(name).cuda().train()
for mod in base.modules():
    if isinstance(mod, torch.nn.Dropout):
        mod.p = 0.0


def run(mode):
    m = copy.deepcopy(base)
    set_backend("native" if mode == "native" else "torch")
    try:
        if mode == "bf16":
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = m(x)
        else:
            out = m(x)
        outs = out if isinstance(out, tuple) else (out,)
        loss = sum(torch.nn.functional.cross_entropy(o.float(), y) for o in outs)
        loss.backward()
    finally:
        set_backend("native")
    return outs[0].detach().float(), {n: p.grad.detach().float().clone() for n, p in m.named_parameters()
                                      if p.grad is not None}


o_n, g_n = run("native")
o_f, g_f = run("fp32")
o_b, g_b = run("bf16")
print(f"{name} bs={bs} size={size} out cos native={cos(o_n, o_f):.5f} torch-bf16={cos(o_b, o_f):.5f}")
names = list(g_f)
worst_n = sorted(names, key=lambda n: cos(g_n[n], g_f[n]))[:8]
for n in names[:6] + worst_n:
    print(f"  {n:45s} native {cos(g_n[n], g_f[n]):8.4f}   torch-bf16 {cos(g_b[n], g_f[n]):8.4f}")
med = lambda d: sorted(cos(d[n], g_f[n]) for n in names)[len(names) // 2]  # noqa: E731
print(f"  median grad cos: native {med(g_n):.4f} torch-bf16 {med(g_b):.4f}")
