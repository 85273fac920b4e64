"""Run-to-run reproducibility of a two-unit ShuffleNet block (default vs deterministic mode):
per-parameter relative gradient differences of repeated fwd+bwd passes from the same weights,
and the gradient at every conv_bn_act input / output (hooks), to find the first op whose result
varies. Run from a tree root (python <path>/diag_shuffle_block.py)."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from deep_vision_amd import set_deterministic  # noqa: E402
from deep_vision_amd.models import mobilenet as MB  # noqa: E402

GRADS = {}
_orig = MB.F.conv_bn_act
_count = [0]


def _keep(k, g):
    GRADS.setdefault(k, g.detach().float().clone())  # returns None: the gradient is not replaced


def hooked(x, conv, bn, *a, **k):
    i = _count[0]
    _count[0] += 1
    if x.requires_grad:
        x.register_hook(lambda g, i=i: _keep(f"{i:02d} in", g))
    y = _orig(x, conv, bn, *a, **k)
    yy = y[0] if isinstance(y, tuple) else y
    yy.register_hook(lambda g, i=i: _keep(f"{i:02d} out", g))
    return y


def unit_forward(self, x):
    """ShuffleUnit.forward with the stride-2 input split per consumer (hooks on each gradient)."""
    F = MB.F
    if self.stride == 2 and os.environ.get("DIAG_SPLIT", "0") == "1":
        xa, xb = x.clone(), x.clone()
        xa.register_hook(lambda g: _keep("u1 x via gconv1", g))
        xb.register_hook(lambda g: _keep("u1 x via avgpool", g))
        y = F.conv_bn_act(xa, self.gconv1, self.bn1, "relu", shuffle=self.groups)
        y.register_hook(lambda g: _keep("u1 bn1 out", g))
        y = F.conv_bn_act(y, self.dwconv, self.bn2, None)
        y = F.conv_bn_act(y, self.gconv2, self.bn3, None)
        sc = F.avg_pool2d(xb, 3, 2, 1)
        sc.register_hook(lambda g: _keep("u1 avgpool out", g))
        return F.relu(F.concat([sc, y]))
    return _orig_unit(self, x)


_orig_unit = MB.ShuffleUnit.forward


def run(mod, x, det):
    GRADS.clear()
    _count[0] = 0
    m = copy.deepcopy(mod).cuda()
    xi = x.clone().requires_grad_(True)
    set_deterministic(det)
    try:
        y = m(xi)
        g = torch.randn(y.shape, device="cuda", generator=torch.Generator(device="cuda").manual_seed(7))
        y.backward(g.to(y.dtype))
        torch.cuda.synchronize()
    finally:
        set_deterministic(False)
    return xi.grad.float(), [(n, p.grad.float().clone()) for n, p in m.named_parameters()], dict(GRADS)


def main():
    if os.environ.get("DIAG_HOOKS", "0") == "1":
        MB.F.conv_bn_act = hooked
    MB.ShuffleUnit.forward = unit_forward
    torch.manual_seed(0)
    mod = torch.nn.Sequential(MB.ShuffleUnit(240, 240, 3, 1), MB.ShuffleUnit(240, 480, 3, 2))
    x = torch.randn(8, 240, 14, 14, device="cuda", generator=torch.Generator(device="cuda").manual_seed(3))
    x = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    rel = lambda u, v: ((u - v).norm() / u.norm().clamp_min(1e-12)).item()  # noqa: E731
    runs = [run(mod, x, d) for d in (False,) * 6 + (True,)]
    for a, b in [(0, 1), (0, 2), (0, 3), (0, 4), (0, 5), (0, 6)]:
        worst = sorted(((rel(u, v), n) for (n, u), (_, v) in zip(runs[a][1], runs[b][1])), reverse=True)[:3]
        print(f"run{a}-run{b}: dx {rel(runs[a][0], runs[b][0]):.2e} worst params",
              ", ".join(f"{n} {r:.2e}" for r, n in worst))
        if runs[a][2]:
            print("   hooks:", ", ".join(f"{k} {rel(runs[a][2][k], runs[b][2][k]):.1e}" for k in sorted(runs[a][2])))


if __name__ == "__main__":
    main()
