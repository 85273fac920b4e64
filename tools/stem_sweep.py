"""Stem conv (ResNet-50 shape: batch 256, 224x224, 7x7/2, 3 -> 64, tap-packed) timing sweep:
forward kernel variants and weight-gradient (variant, split %) pairs.
python tools/stem_sweep.py [--fwd 0,1,...] [--wg 0,2,4,6] [--splits 50,100,200,400]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_vision_amd import ops as F  # noqa: E402
from deep_vision_amd._ext import lib  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fwd", default="0")
    ap.add_argument("--wg", default="0")
    ap.add_argument("--splits", default="100")
    ap.add_argument("--det", action="store_true", help="deterministic slab split-K (plain stores + ordered reduce)")
    a = ap.parse_args()
    if a.det:
        lib().set_deterministic(True)
    x = torch.randn(256, 3, 224, 224, device="cuda")
    w = (torch.randn(64, 3, 7, 7, device="cuda") * 0.05).requires_grad_(True)
    flops = 2.0 * 256 * 112 * 112 * 64 * 147
    ref = None
    for v in [int(s) for s in a.fwd.split(",")]:
        lib().conv_fwd_variant(v)
        y = F.conv2d(x, w, None, 2, 3)
        torch.cuda.synchronize()
        ref = y.float() if ref is None else ref
        err = float((y.float() - ref).abs().max())
        us = timeit(lambda: F.conv2d(x, w, None, 2, 3))
        print(f"fwd v{v}: {us:8.1f} us (incl. pack) {flops / us / 1e6:7.1f} TF/s maxdiff {err:.3g}", flush=True)
    lib().conv_fwd_variant(0)
    y = F.conv2d(x, w, None, 2, 3)
    g = torch.randn_like(y)
    gref = None
    for v in [int(s) for s in a.wg.split(",")]:
        for sp in [int(s) for s in a.splits.split(",")]:
            lib().conv_wgrad_tuning(v, sp)
            (dw,) = torch.autograd.grad(y, w, g, retain_graph=True)
            torch.cuda.synchronize()
            gref = dw if gref is None else gref
            err = float((dw - gref).abs().max() / gref.abs().max())
            us = timeit(lambda: torch.autograd.grad(y, w, g, retain_graph=True))
            print(f"wgrad v{v} split {sp:4d}%: {us:8.1f} us {flops / us / 1e6:7.1f} TF/s relerr {err:.3g}", flush=True)
    lib().conv_wgrad_tuning(0, 100)


if __name__ == "__main__":
    main()
