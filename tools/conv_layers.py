"""Per-layer conv table of a zoo model at its bench batch: native implicit-GEMM kernels vs MIOpen,
forward / dgrad / wgrad (YOLOv3's Darknet-53 + head shapes, the Keras
asymmetric stride-2 3x3s and the 13x13 K = 4608 layers).

python tools/conv_layers.py --model yolov3 [--batch 16] [--size 416] [--iters 20] [--out FILE]

The layer list comes from the model itself: every ops.conv.conv2d call of one forward is recorded
(Cin, Cout, H, W, k, stride, padding); identical shapes are merged with their count. Native: ops.conv.conv2d (forward, weight cache warm), ops.conv._dgrad and _wgrad (the
autograd backward's own calls). MIOpen: torch conv2d / aten.convolution_backward on bf16
channels-last tensors (asymmetric 'same' padding as an explicit pad of the input: included in its
time). Small layers are host-issue-bound here (eager, one call per timing iteration); the captured
step (bench.py --graph) does not pay that.
"""
from __future__ import annotations

import argparse
import os
import sys

import torch
import torch.nn.functional as TF

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from conv_vs_miopen import timeit  # noqa: E402

from deep_vision_amd import models as M  # noqa: E402
from deep_vision_amd.ops.conv import _dgrad, _wgrad, conv2d, norm_padding  # noqa: E402

CL = torch.channels_last


def collect(model, x):
    """Every ops.conv.conv2d call of one forward (the fused conv -> BN paths call it directly, not
    through the module): (Cin, Cout, H, W, k, stride, padding, groups) -> count."""
    from deep_vision_amd.ops import conv as C

    seen = {}
    inner = C.conv2d

    def rec(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, *a, **k):
        s = stride if isinstance(stride, int) else stride[0]
        pad = tuple(padding) if not isinstance(padding, int) else (padding, padding)
        key = (x.shape[1], weight.shape[0], x.shape[2], x.shape[3], weight.shape[2], s, pad, groups)
        seen[key] = seen.get(key, 0) + 1
        return inner(x, weight, bias, stride, padding, dilation, groups, *a, **k)

    C.conv2d = rec
    try:
        with torch.no_grad():
            model(x)
    finally:
        C.conv2d = inner
    return seen


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="yolov3")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=416)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda")
    kw = {"hourglass104": dict(num_stack=4, num_residual=1, num_heatmap=16)}.get(a.model, {})  # bench.py's configs
    model = M.get_model(a.model, **kw).to(dev)
    x0 = torch.randn(a.batch, 3, a.size, a.size, device=dev)
    layers = collect(model, x0)
    del model
    N = a.batch
    hdr = (f"{'layer':>34s} {'x':>2s} | {'fwd us':>8s} {'miopen':>8s} {'TF/s':>6s} | {'dgrad':>8s} {'miopen':>8s} "
           f"{'TF/s':>6s} | {'wgrad':>8s} {'miopen':>8s} {'TF/s':>6s}")
    lines = [hdr]
    print(hdr, flush=True)
    tot = {"native": [0.0, 0.0, 0.0], "miopen": [0.0, 0.0, 0.0]}
    flop_tot = 0.0
    for (cin, cout, H, W, k, s, pad, groups), cnt in sorted(layers.items(), key=lambda kv: (-kv[0][2], kv[0][0])):
        if groups != 1 or cin < 8:
            continue  # the stem (tap-packed path) and grouped convs are not GEMM-table shapes
        (pt, pl), (eb, er) = norm_padding(pad if len(pad) == 4 else (pad[0], pad[0], pad[1], pad[1]))
        P = (H + pt + pt + eb - k) // s + 1
        Q = (W + pl + pl + er - k) // s + 1
        x = torch.randn(N, cin, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
        w = torch.nn.Parameter(torch.randn(cout, cin, k, k, device=dev) * (2.0 / (cin * k * k)) ** 0.5)
        # an output channel count that is not a multiple of 8 lives in a padded NHWC buffer, as in
        # the model (ops.conv returns a channel-slice view of it)
        dy = torch.randn(N, -(-cout // 8) * 8, P, Q, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)[:, :cout]
        wb = w.detach().to(torch.bfloat16).contiguous(memory_format=CL)
        gw = torch.zeros_like(w)
        flop = 2.0 * N * P * Q * cout * cin * k * k
        mpad = (pl, pl + er, pt, pt + eb)
        xm = TF.pad(x, mpad) if (eb or er) else x
        mp = 0 if (eb or er) else pt
        with torch.no_grad():
            t_nf = timeit(lambda: conv2d(x, w, None, s, pad), a.iters)
            t_nd = timeit(lambda: _dgrad(dy, w, x.shape, cin, 1, (s, s), (pt, pl), (1, 1), dev), a.iters)
            t_nw = timeit(lambda: _wgrad(x, dy, w, cin, 1, (s, s), (pt, pl), (1, 1), out=gw), a.iters)
            t_mf = timeit(lambda: TF.conv2d(TF.pad(x, mpad) if (eb or er) else x, wb, None, s, mp), a.iters)
            t_md = timeit(lambda: torch.ops.aten.convolution_backward(dy, xm, wb, None, [s, s], [mp, mp], [1, 1], False,
                                                                      [0, 0], 1, [True, False, False]), a.iters)
            t_mw = timeit(lambda: torch.ops.aten.convolution_backward(dy, xm, wb, None, [s, s], [mp, mp], [1, 1], False,
                                                                      [0, 0], 1, [False, True, False]), a.iters)
        name = f"{cin:5d}->{cout:5d} @{H:3d}x{W:<3d} k{k} s{s}" + ("*" if (eb or er) else " ")
        ln = (f"{name:>34s} {cnt:2d} | {t_nf:8.1f} {t_mf:8.1f} {flop / t_nf / 1e6:6.0f} | {t_nd:8.1f} {t_md:8.1f} "
              f"{flop / t_nd / 1e6:6.0f} | {t_nw:8.1f} {t_mw:8.1f} {flop / t_nw / 1e6:6.0f}")
        print(ln, flush=True)
        lines.append(ln)
        flop_tot += 3 * cnt * flop
        for i, (tn, tm) in enumerate(((t_nf, t_mf), (t_nd, t_md), (t_nw, t_mw))):
            tot["native"][i] += cnt * tn
            tot["miopen"][i] += cnt * tm
    for arm, v in tot.items():
        ln = (f"per-step total ({arm}, weighted by count, stem excluded): fwd {v[0] / 1e3:.2f} ms  dgrad "
              f"{v[1] / 1e3:.2f} ms  wgrad {v[2] / 1e3:.2f} ms  sum {sum(v) / 1e3:.2f} ms  "
              f"({flop_tot / sum(v) / 1e6:.0f} TF/s over {flop_tot / 1e12:.2f} TFLOP)")
        print(ln, flush=True)
        lines.append(ln)
    lines.append("* Keras 'same' padding with an extra bottom/right row (stride 2): the native gather reads it as "
                 "zeros; MIOpen pads the input first (in its time)")
    if a.out:
        with open(a.out, "w") as f:
            f.write(f"# tools/conv_layers.py --model {a.model} --batch {N} --size {a.size} --iters {a.iters} "
                    "(1x MI355X; TF/s = native)\n")
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
