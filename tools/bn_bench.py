"""Microbenchmark of the BN backward-reduce pass at the ResNet-50 (batch 256) shapes: grid size
and loop unroll variants, interleaved rounds in one process (cdna_hip_programming §5.4 rule 24).

usage: python tools/bn_bench.py [--iters 20] [--rounds 3]
"""
import argparse
import sys

import torch

sys.path.insert(0, ".")
from deep_vision_amd._ext import lib, ptr, stream_handle  # noqa: E402

SHAPES = [  # (name, rows, C, mask mode) mask: "bits" (residual BN3) | "x" (BN1/BN2, mask recomputed from x)
    ("c3_256@56", 256 * 56 * 56, 256, "bits"),
    ("c1_64@56", 256 * 56 * 56, 64, "x"),
    ("c3_512@28", 256 * 28 * 28, 512, "bits"),
    ("c1_128@28", 256 * 28 * 28, 128, "x"),
    ("c3_1024@14", 256 * 14 * 14, 1024, "bits"),
    ("c1_256@14", 256 * 14 * 14, 256, "x"),
    ("c3_2048@7", 256 * 7 * 7, 2048, "bits"),
]
VARIANTS = [(1024, 2), (2048, 2), (1024, 4), (2048, 4), (4096, 4), (512, 4)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    L = lib()
    st = stream_handle()
    for name, rows, C, mm in SHAPES:
        d = torch.randn(rows, C, device="cuda").bfloat16()
        x = torch.randn(rows, C, device="cuda").bfloat16()
        bits = torch.randint(0, 255, (rows * C // 8,), dtype=torch.uint8, device="cuda") if mm == "bits" else None
        prm = torch.randn(4, C, device="cuda")
        acc = torch.zeros(64, 2, C, device="cuda")
        nbytes = 2 * rows * C * 2 + (rows * C // 8 if bits is not None else 0)
        res = {v: [] for v in VARIANTS}
        for _ in range(a.rounds):
            for v in VARIANTS:
                L.bn_tuning(*v)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                for it in range(a.iters + 2):
                    if it == 2:
                        e0.record()
                    L.bn_bwd_reduce(ptr(d), ptr(bits) if bits is not None else 0, ptr(x), rows, C, ptr(prm[0]),
                                    ptr(prm[1]), ptr(prm[2]), ptr(prm[3]), 1, 0.0, ptr(acc),
                                    int(bits is not None), st)
                e1.record()
                torch.cuda.synchronize()
                res[v].append(e0.elapsed_time(e1) / a.iters * 1e3)
        L.bn_tuning(0, 0)
        for v in VARIANTS:
            t = min(res[v])
            print(f"{name:12s} blocks={v[0]:5d} unroll={v[1]}  {t:8.1f} us  {nbytes / t / 1e3:7.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
