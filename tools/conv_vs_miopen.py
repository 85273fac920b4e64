"""Per-layer ResNet-50 conv table: native implicit-GEMM kernels vs MIOpen (PyTorch's bf16 NHWC
convolution on ROCm), forward / dgrad / wgrad, at the bench batch.

python tools/conv_vs_miopen.py [--batch 256] [--iters 20] [--out profiles/conv_bench_resnet50_vs_miopen.txt]

Native: the production entry points (ops.conv.conv2d forward with the weight cache warm,
ops.conv._dgrad, ops.conv._wgrad into an fp32 gradient). MIOpen: torch.nn.functional.conv2d and
aten.convolution_backward (input-only / weight-only masks) on bf16 channels-last tensors with
bf16 weights. Layer multiplicities are the ResNet-50 counts (R/ResNet/pytorch/models/resnet50.py:101-133).
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_vision_amd.ops.conv import _dgrad, _wgrad, conv2d  # noqa: E402

CL = torch.channels_last
# (Cin, Cout, H_in, k, stride, count per step): stride on the first 1x1 of a stage (ResNet V1)
LAYERS = [
    (64, 64, 56, 1, 1, 1), (256, 64, 56, 1, 1, 2), (64, 64, 56, 3, 1, 3), (64, 256, 56, 1, 1, 4),
    (256, 128, 56, 1, 2, 1), (256, 512, 56, 1, 2, 1), (128, 128, 28, 3, 1, 4), (128, 512, 28, 1, 1, 4),
    (512, 128, 28, 1, 1, 3),
    (512, 256, 28, 1, 2, 1), (512, 1024, 28, 1, 2, 1), (256, 256, 14, 3, 1, 6), (256, 1024, 14, 1, 1, 6),
    (1024, 256, 14, 1, 1, 5),
    (1024, 512, 14, 1, 2, 1), (1024, 2048, 14, 1, 2, 1), (512, 512, 7, 3, 1, 3), (512, 2048, 7, 1, 1, 3),
    (2048, 512, 7, 1, 1, 2),
]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000.0 / iters  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True  # MIOpen: find the best solver per shape first
    N = a.batch
    dev = torch.device("cuda")
    lines = []
    tot = {"native": [0.0, 0.0, 0.0], "miopen": [0.0, 0.0, 0.0]}
    hdr = (f"{'layer':>26s} {'x':>2s} | {'fwd us':>8s} {'miopen':>8s} {'TF/s':>6s} | {'dgrad':>8s} {'miopen':>8s} "
           f"{'TF/s':>6s} | {'wgrad':>8s} {'miopen':>8s} {'TF/s':>6s}")
    print(hdr, flush=True)
    lines.append(hdr)
    for cin, cout, H, k, s, cnt in LAYERS:
        p = k // 2
        P = (H + 2 * p - k) // s + 1
        x = torch.randn(N, cin, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
        w = torch.nn.Parameter(torch.randn(cout, cin, k, k, device=dev) * (2.0 / (cin * k * k)) ** 0.5)
        dy = torch.randn(N, cout, P, P, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
        wb = w.detach().to(torch.bfloat16).contiguous(memory_format=CL)
        gw = torch.zeros_like(w)
        flop = 2.0 * N * P * P * cout * cin * k * k
        with torch.no_grad():
            t_nf = timeit(lambda: conv2d(x, w, None, s, p), a.iters)
            t_nd = timeit(lambda: _dgrad(dy, w, x.shape, cin, 1, (s, s), (p, p), (1, 1), dev), a.iters)
            t_nw = timeit(lambda: _wgrad(x, dy, w, cin, 1, (s, s), (p, p), (1, 1), out=gw), a.iters)
            t_mf = timeit(lambda: torch.nn.functional.conv2d(x, wb, None, s, p), a.iters)
            t_md = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, wb, None, [s, s], [p, p], [1, 1], False,
                                                                      [0, 0], 1, [True, False, False]), a.iters)
            t_mw = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, wb, None, [s, s], [p, p], [1, 1], False,
                                                                      [0, 0], 1, [False, True, False]), a.iters)
        name = f"{cin:5d}->{cout:5d} @{H:3d} k{k} s{s}"
        ln = (f"{name:>26s} {cnt:2d} | {t_nf:8.1f} {t_mf:8.1f} {flop / t_nf / 1e6:6.0f} | {t_nd:8.1f} {t_md:8.1f} "
              f"{flop / t_nd / 1e6:6.0f} | {t_nw:8.1f} {t_mw:8.1f} {flop / t_nw / 1e6:6.0f}")
        print(ln, flush=True)
        lines.append(ln)
        for i, (tn, tm) in enumerate(((t_nf, t_mf), (t_nd, t_md), (t_nw, t_mw))):
            tot["native"][i] += cnt * tn
            tot["miopen"][i] += cnt * tm
    for arm, v in tot.items():
        ln = (f"per-step total ({arm}, weighted by count, stem excluded): fwd {v[0] / 1e3:.2f} ms  dgrad "
              f"{v[1] / 1e3:.2f} ms  wgrad {v[2] / 1e3:.2f} ms  sum {sum(v) / 1e3:.2f} ms")
        print(ln, flush=True)
        lines.append(ln)
    if a.out:
        with open(a.out, "w") as f:
            f.write(f"# tools/conv_vs_miopen.py --batch {N} --iters {a.iters} (1x MI355X; TF/s = native)\n")
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
