#!/usr/bin/env python3
"""Per-layer conv microbenchmark: native gfx950 implicit GEMM vs PyTorch/MIOpen on the same box.

Times forward, dgrad and wgrad of every unique ResNet-50 conv shape at the
benchmark batch, interleaving native and MIOpen rounds in one process (methodology rule 24),
and prints TFLOP/s per pass plus the per-step total weighted by layer multiplicity.

    python bench/conv_bench.py [--batch 256] [--iters 20] [--only fwd|dgrad|wgrad] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (Cin, Cout, H, R, stride, pad, count in ResNet-50)
RESNET50_SHAPES = [
    (3, 64, 224, 7, 2, 3, 1),
    (64, 64, 56, 1, 1, 0, 1), (64, 64, 56, 3, 1, 1, 3), (64, 256, 56, 1, 1, 0, 4), (256, 64, 56, 1, 1, 0, 2),
    (256, 128, 56, 1, 2, 0, 1), (128, 128, 28, 3, 1, 1, 4), (128, 512, 28, 1, 1, 0, 4), (256, 512, 56, 1, 2, 0, 1),
    (512, 128, 28, 1, 1, 0, 3),
    (512, 256, 28, 1, 2, 0, 1), (256, 256, 14, 3, 1, 1, 6), (256, 1024, 14, 1, 1, 0, 6), (512, 1024, 28, 1, 2, 0, 1),
    (1024, 256, 14, 1, 1, 0, 5),
    (1024, 512, 14, 1, 2, 0, 1), (512, 512, 7, 3, 1, 1, 3), (512, 2048, 7, 1, 1, 0, 3), (1024, 2048, 14, 1, 2, 0, 1),
    (2048, 512, 7, 1, 1, 0, 2),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default=None)
    ap.add_argument("--json", default=None)
    ap.add_argument("--no-torch", action="store_true")
    a = ap.parse_args()

    import torch
    import torch.nn.functional as TF

    from deep_vision_amd.ops import conv as C
    from deep_vision_amd.ops.common import as_nhwc

    dev = torch.device("cuda")
    torch.backends.cudnn.benchmark = True
    N = a.batch
    results = []
    tot = {"native": {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}, "torch": {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}}

    def timeit(fn, iters):
        for _ in range(3):
            fn()
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / iters * 1e3  # us

    for (cin, cout, H, R, st, pd, cnt) in RESNET50_SHAPES:
        P = (H + 2 * pd - R) // st + 1
        x32 = torch.randn(N, cin, H, H, device=dev)
        w = torch.randn(cout, cin, R, R, device=dev) * 0.05
        x = as_nhwc(x32)
        flops = 2.0 * N * P * P * cout * cin * R * R
        y = C.conv2d(x, w, None, st, pd)
        dy = torch.randn_like(y.float()).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        Cg = C._gather_channels(x, cin, 1)
        row = {"shape": [cin, cout, H, R, st], "count": cnt, "gflop": flops / 1e9}
        passes = {
            "fwd": lambda: C.conv2d(x, w, None, st, pd),
            "dgrad": lambda: C._dgrad(dy, w, x.shape, Cg, 1, (st, st), (pd, pd), (1, 1), dev),
            "wgrad": lambda: C._wgrad(x, dy, w, Cg, 1, (st, st), (pd, pd), (1, 1)),
        }
        xt = x32.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wt = w.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dyt = dy
        tpasses = {
            "fwd": lambda: TF.conv2d(xt, wt, None, st, pd),
            "dgrad": lambda: torch.ops.aten.convolution_backward(dyt, xt, wt, None, (st, st), (pd, pd), (1, 1), False,
                                                                 (0, 0), 1, (True, False, False)),
            "wgrad": lambda: torch.ops.aten.convolution_backward(dyt, xt, wt, None, (st, st), (pd, pd), (1, 1), False,
                                                                 (0, 0), 1, (False, True, False)),
        }
        for k in ("fwd", "dgrad", "wgrad"):
            if a.only and k != a.only:
                continue
            if k == "dgrad" and cin == 3:
                continue
            tn = timeit(passes[k], a.iters)
            tt = timeit(tpasses[k], a.iters) if not a.no_torch else float("nan")
            row[k] = {"native_us": round(tn, 1), "torch_us": round(tt, 1), "native_tflops": round(flops / tn / 1e6, 1),
                      "torch_tflops": round(flops / tt / 1e6, 1) if tt == tt else None}
            tot["native"][k] += tn * cnt
            if tt == tt:
                tot["torch"][k] += tt * cnt
        results.append(row)
        line = f"{cin:5d}->{cout:5d} {H:4d} k{R} s{st} x{cnt}: " + "  ".join(
            f"{k} {row[k]['native_us']:8.1f}us ({row[k]['native_tflops']:6.1f}TF) vs miopen {row[k]['torch_us']:8.1f}us"
            for k in ("fwd", "dgrad", "wgrad") if k in row)
        print(line, flush=True)
    print("per-step totals (us, weighted by multiplicity):")
    for be in ("native", "torch"):
        print(f"  {be:7s} " + "  ".join(f"{k}={v/1e3:.2f}ms" for k, v in tot[be].items()) +
              f"  sum={sum(tot[be].values())/1e3:.2f}ms")
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"batch": N, "layers": results, "totals_us": tot}, f, indent=1)


if __name__ == "__main__":
    main()
