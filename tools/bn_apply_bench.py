"""Microbenchmark of the BN apply passes at the ResNet-50 (batch 256) shapes: the block-output
forward apply (x*scale + shift + residual, ReLU, mask bits) and the residual BN backward apply
(mask bits), over (grid blocks, rows in flight per thread) variants in interleaved rounds.

usage: python tools/bn_apply_bench.py [--iters 20] [--rounds 3]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_vision_amd._ext import lib, ptr, stream_handle  # noqa: E402

SHAPES = [("256@56", 256 * 56 * 56, 256), ("512@28", 256 * 28 * 28, 512), ("1024@14", 256 * 14 * 14, 1024),
          ("2048@7", 256 * 7 * 7, 2048), ("64@56", 256 * 56 * 56, 64)]
VARIANTS = [(0, 2), (8192, 2), (16384, 2), (8192, 4)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    L, st = lib(), stream_handle()
    for name, rows, C in SHAPES:
        n = rows * C
        x = torch.randn(n, device="cuda").bfloat16()
        r = torch.randn(n, device="cuda").bfloat16()
        out = torch.empty_like(x)
        bits = torch.empty(n // 8, dtype=torch.uint8, device="cuda")
        sc, sh = torch.rand(C, device="cuda"), torch.randn(C, device="cuda")
        x2, out2 = torch.randn(n, device="cuda").bfloat16(), torch.empty_like(out)
        k = torch.rand(3, C, device="cuda")
        ops = {
            "fwd_apply+res+bits": (lambda: L.bn_apply(ptr(x), ptr(r), ptr(out), n, C, ptr(sc), ptr(sh), 1, 0.0, ptr(bits), st),
                                   n * 6 + n // 8),
            "bwd_apply bits": (lambda: L.bn_bwd_apply(ptr(x), ptr(bits), ptr(r), ptr(out), 0, n, C, ptr(sc), ptr(sh), ptr(sc),
                                                      0, 0, 1, 0.0, 1, st), n * 6 + n // 8),
            # both BNs of a projection block's join: dout, bits, x, x2 in; dx, dx2 out
            "bwd_apply_dual": (lambda: L.bn_bwd_apply_dual(ptr(x), ptr(bits), ptr(r), ptr(x2), ptr(out), ptr(out2), n, C,
                                                           ptr(k), ptr(k), 1, 0.0, st), n * 10 + n // 8),
        }
        for oname, (fn, nbytes) in ops.items():
            res = {v: [] for v in VARIANTS}
            for _ in range(a.rounds):
                for v in VARIANTS:
                    L.bn_apply_tuning(*v)
                    fn()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(a.iters):
                        fn()
                    e1.record()
                    torch.cuda.synchronize()
                    res[v].append(e0.elapsed_time(e1) / a.iters * 1e3)
            for v, ts in res.items():
                us = min(ts)
                print(f"{name:8s} {oname:20s} blocks={v[0]:5d} unroll={v[1]}  {us:8.1f} us  {nbytes / us / 1e3:6.0f} GB/s",
                      flush=True)
    L.bn_apply_tuning(0, 2)


if __name__ == "__main__":
    main()
