"""Cost of the fused dgrad epilogues (csrc/conv_fwd.hip): the 1x1 dgrad of a bottleneck's first
conv on the ResNet-50 shapes, plain vs + residual-gradient join (masked by the block's ReLU bits)
vs + BatchNorm-backward statistics of the upstream BN (bnmode 3) vs both, as in the training step.

usage: python tools/epi_bench.py [--iters 20]
"""
import argparse
import os
import sys
from types import SimpleNamespace

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_vision_amd.ops.conv import conv_fwd_raw  # noqa: E402

CL = torch.channels_last
# (name, batch, H, K = dY channels, N = dX channels): dgrad of the block's 1x1 conv1 (N -> K)
SHAPES = [("s1", 256, 56, 64, 256), ("s2", 256, 28, 128, 512), ("s3", 256, 14, 256, 1024), ("s4", 256, 7, 512, 2048)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    for name, Nb, H, K, N in SHAPES:
        M = Nb * H * H
        dy = torch.randn(Nb, K, H, H, device="cuda").bfloat16().contiguous(memory_format=CL)
        wk = (torch.randn(N, K, device="cuda") * 0.05).bfloat16().contiguous()
        dx = torch.empty(Nb, N, H, H, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=CL)
        res = torch.randn(Nb, N, H, H, device="cuda").bfloat16().contiguous(memory_format=CL)
        bits = torch.randint(0, 255, (M * N // 8,), device="cuda", dtype=torch.uint8)
        bnx = torch.randn(Nb, N, H, H, device="cuda").bfloat16().contiguous(memory_format=CL)
        prm = torch.rand(4, N, device="cuda")
        acc = torch.zeros(64, 2, N, device="cuda")
        ref = SimpleNamespace(x=bnx, bits=bits, prm=prm, acc=acc, mode=3, act=1, slope=0.0)
        cases = {
            "plain": dict(),
            "res": dict(res=res, resmask=(bits, 1, 0.0)),
            "bnr": dict(bnref=ref),
            "res+bnr": dict(res=res, resmask=(bits, 1, 0.0), bnref=ref),
        }
        flops = 2.0 * M * N * K
        for cname, kw in cases.items():
            def fn():
                conv_fwd_raw(dy, wk, dx, None, None, Nb, H, H, K, K, 1, N, H, H, 1, 1, (1, 1), (0, 0), (1, 1), **kw)
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / a.iters * 1e3
            nb = M * K * 2 + M * N * 2 * (1 + ("res" in cname) + ("bnr" in cname)) + M * N / 8 * (cname != "plain")
            print(f"{name} M={M:7d} K={K:4d} N={N:5d} {cname:8s} {us:8.1f} us  {flops / us / 1e6:6.0f} TF  "
                  f"{nb / us / 1e3:6.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
