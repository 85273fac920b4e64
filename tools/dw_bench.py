"""Depthwise conv kernels (fwd / dgrad / wgrad) on the MobileNet V1 layer shapes at batch 128:
every variant (csrc/depthwise.hip g_dw_variant) in interleaved rounds, checked against variant 0,
with effective HBM bandwidth (minimum bytes: read input(s) once, write output once).

usage: python tools/dw_bench.py [--variants 0,1,2,3,4,5] [--iters 10]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_vision_amd._ext import lib, ptr, stream_handle  # noqa: E402

CL = torch.channels_last
# (C, H_in, stride) of the 13 depthwise layers of MobileNet V1 at 224
LAYERS = [(32, 112, 1), (64, 112, 2), (128, 56, 1), (128, 56, 2), (256, 28, 1), (256, 28, 2), (512, 14, 1),
          (512, 14, 2), (1024, 7, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1,2,3,4,5")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--stats", action="store_true", help="forward with fused BN statistics (MobileNet's form)")
    a = ap.parse_args()
    vs = [int(v) for v in a.variants.split(",")]
    L = lib()
    st = stream_handle()
    N = a.batch
    for C, H, s in LAYERS:
        P = (H + 2 - 3) // s + 1
        x = torch.randn(N, C, H, H, device="cuda").bfloat16().contiguous(memory_format=CL)
        dy = torch.randn(N, C, P, P, device="cuda").bfloat16().contiguous(memory_format=CL)
        w = torch.randn(C, 1, 3, 3, device="cuda") * 0.3
        y = torch.empty(N, C, P, P, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=CL)
        dx = torch.empty_like(x)
        dw = torch.zeros(C, 9, device="cuda")
        acc = torch.zeros(129 * C, device="cuda")  # [64][2][C] shards + the shift row
        sp = ptr(acc) if a.stats else 0
        bx, by = x.numel() * 2, y.numel() * 2
        ops = {
            "fwd": (lambda: L.dw_fwd(ptr(x), ptr(w), 0, ptr(y), N, H, H, C, C, P, P, C, 3, s, s, 1, 1, 0, 0.0, sp, st),
                    y, bx + by),
            "dgrad": (lambda: L.dw_dgrad(ptr(dy), ptr(w), ptr(dx), N, H, H, C, C, P, P, C, 3, s, s, 1, 1, st), dx,
                      bx + by),
            "wgrad": (lambda: L.dw_wgrad(ptr(x), ptr(dy), ptr(dw), N, H, H, C, C, P, P, C, 3, s, s, 1, 1, 0, st), dw,
                      bx + by),
        }
        for name, (fn, out, nbytes) in ops.items():
            ref = None
            res = {v: [] for v in vs}
            for rnd in range(2):
                for v in vs:
                    L.dw_variant(v)
                    fn()
                    torch.cuda.synchronize()
                    if v == vs[0] and ref is None:
                        ref = out.float().clone()
                    err = ((out.float() - ref).abs().max() / ref.abs().max().clamp_min(1e-20)).item()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(a.iters):
                        fn()
                    e1.record()
                    torch.cuda.synchronize()
                    res[v].append((e0.elapsed_time(e1) * 1e3 / a.iters, err))
            L.dw_variant(0)
            for v in vs:
                us = min(t for t, _ in res[v])
                err = max(e for _, e in res[v])
                print(f"{name:5s} C{C:5d} H{H:4d} s{s}  v{v}  {us:8.1f} us  {nbytes / us / 1e3:7.0f} GB/s  relerr {err:.2e}",
                      flush=True)


if __name__ == "__main__":
    main()
