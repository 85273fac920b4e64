"""Grouped 1x1 kernels (csrc/gconv.hip) on the ShuffleNet V1 g=3 layer shapes at batch 128:
fwd / dgrad / wgrad time and effective HBM bandwidth (inputs read once + output written once).

usage: python tools/gconv_bench.py [--iters 20] [--batch 128]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_vision_amd._ext import lib, ptr, stream_handle  # noqa: E402
from deep_vision_amd.ops.conv import _shuffle_table  # noqa: E402

CL = torch.channels_last
# (Cin, Cout, G, shuffle, H) of ShuffleNet V1 1x g=3 at 224 (one of each distinct shape)
LAYERS = [(24, 60, 1, 3, 56), (60, 216, 3, 0, 28), (240, 60, 3, 3, 28), (60, 240, 3, 0, 28),
          (240, 120, 3, 3, 28), (120, 240, 3, 0, 14), (480, 120, 3, 3, 14), (120, 480, 3, 0, 14),
          (480, 240, 3, 3, 14), (240, 480, 3, 0, 7), (960, 240, 3, 3, 7), (240, 960, 3, 0, 7)]


def r8(v):
    return (v + 7) // 8 * 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=128)
    a = ap.parse_args()
    L, st, N = lib(), stream_handle(), a.batch
    for Cin, Cout, G, sg, H in LAYERS:
        M = N * H * H
        Cg, Og = Cin // G, Cout // G
        x = torch.randn(M, r8(Cin), device="cuda").bfloat16()
        dy = torch.randn(M, r8(Cout), device="cuda").bfloat16()
        y = torch.empty(M, r8(Cout), device="cuda", dtype=torch.bfloat16)
        dx = torch.empty(M, r8(Cin), device="cuda", dtype=torch.bfloat16)
        Kp, Kq = (Cg + 31) // 32 * 32, (Og + 31) // 32 * 32
        wk = torch.randn(G, Og, Kp, device="cuda").bfloat16()
        wt = torch.randn(G, Cg, Kq, device="cuda").bfloat16()
        dw = torch.zeros(Cout, Cg, device="cuda")
        tab = _shuffle_table(Cout, sg, x.device)
        bx, by = M * Cin * 2, M * Cout * 2
        ops = {
            "fwd": (lambda: L.gconv(ptr(x), r8(Cin), Cin, 0, ptr(wk), Og, ptr(y), r8(Cout), Cout, ptr(tab), M, G, Cg, Og,
                                    Kp, 0, st), bx + by),
            "dgrad": (lambda: L.gconv(ptr(dy), r8(Cout), Cout, ptr(tab), ptr(wt), Cg, ptr(dx), r8(Cin), Cin, 0, M, G, Og,
                                      Cg, Kq, 0, st), bx + by),
            "wgrad": (lambda: L.gconv_wgrad(ptr(x), r8(Cin), 0, ptr(dy), r8(Cout), ptr(tab), ptr(dw), M, G, Cg, Og, st),
                      bx + by),
        }
        for name, (fn, nbytes) in ops.items():
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / a.iters * 1e3
            print(f"{name:5s} {Cin:4d}->{Cout:4d} g{G} sh{sg} @{H:3d}  {us:8.1f} us  {nbytes / us / 1e3:7.0f} GB/s",
                  flush=True)


if __name__ == "__main__":
    main()
