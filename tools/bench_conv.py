"""Micro-benchmark of the implicit-GEMM forward / wgrad kernel variants on ResNet-50 layer shapes.

python tools/bench_conv.py [--batch 256] [--variants 0,1,2,...]
Runs every (layer, variant) on the GPU, checks each variant's output against variant 0
(bit-exact up to accumulation order) and prints us / TFLOP/s / effective GB/s. Variant ids:
csrc/conv_fwd.hip dispatch_res (0 = heuristic).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from deep_vision_amd._ext import lib
from deep_vision_amd.ops.conv import conv_fwd_raw

CL = torch.channels_last

# (name, H, Cin, Cout, k, stride)  -- forward convs of ResNet-50 at 224
LAYERS = [
    ("s1_1x1_64_64", 56, 64, 64, 1, 1), ("s1_3x3_64", 56, 64, 64, 3, 1), ("s1_1x1_64_256", 56, 64, 256, 1, 1),
    ("s1_1x1_256_64", 56, 256, 64, 1, 1),
    ("s2_1x1_256_128", 56, 256, 128, 1, 1), ("s2_3x3_128_s2", 56, 128, 128, 3, 2), ("s2_3x3_128", 28, 128, 128, 3, 1),
    ("s2_1x1_128_512", 28, 128, 512, 1, 1), ("s2_1x1_512_128", 28, 512, 128, 1, 1), ("s2_proj_256_512_s2", 56, 256, 512, 1, 2),
    ("s3_3x3_256", 14, 256, 256, 3, 1), ("s3_1x1_256_1024", 14, 256, 1024, 1, 1), ("s3_1x1_1024_256", 14, 1024, 256, 1, 1),
    ("s4_3x3_512", 7, 512, 512, 3, 1), ("s4_1x1_512_2048", 7, 512, 2048, 1, 1), ("s4_1x1_2048_512", 7, 2048, 512, 1, 1),
    # dgrad shapes (forward kernel on dY with the transposed weights)
    ("dg_s1_256_to_64", 56, 256, 64, 1, 1), ("dg_s1_64_to_256", 56, 64, 256, 1, 1),
    ("dg_s3_1024_to_256", 14, 1024, 256, 1, 1),
]


# Stacked Hourglass (batch 32) bottleneck convs at the 64x64 and 32x32 scales
HOURGLASS = [
    ("hg64_1x1_256_128", 64, 256, 128, 1, 1), ("hg64_3x3_128", 64, 128, 128, 3, 1), ("hg64_1x1_128_256", 64, 128, 256, 1, 1),
    ("hg32_1x1_256_128", 32, 256, 128, 1, 1), ("hg32_3x3_128", 32, 128, 128, 3, 1), ("hg32_1x1_128_256", 32, 128, 256, 1, 1),
    ("hg16_3x3_128", 16, 128, 128, 3, 1), ("hg8_3x3_128", 8, 128, 128, 3, 1),
]

# YOLOv3 (batch 16, 416) Darknet-53 3x3 convs at the under-filled 13x13 / 26x26 scales
YOLOV3 = [
    ("yl13_3x3_512_1024", 13, 512, 1024, 3, 1), ("yl26_3x3_256_512", 26, 256, 512, 3, 1),
    ("yl52_3x3_128_256", 52, 128, 256, 3, 1), ("yl13_1x1_1024_512", 13, 1024, 512, 1, 1),
]


def run(name, H, Cin, Cout, k, s, N, variants, iters, ksplits=(1,)):
    pad = k // 2
    P = (H + 2 * pad - k) // s + 1
    x = torch.randn(N, Cin, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(Cout, k, k, Cin, device="cuda") * 0.05).to(torch.bfloat16).contiguous()
    y = torch.empty(N, Cout, P, P, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=CL)
    flops = 2.0 * N * P * P * Cout * Cin * k * k
    nbytes = 2.0 * (N * H * H * Cin + N * P * P * Cout)
    res, ref = {}, None
    for v, ks in [(v, ks) for v in variants for ks in ksplits]:
        lib().conv_fwd_variant(v)

        def go():
            conv_fwd_raw(x, w, y, None, None, N, H, H, Cin, Cin, 1, Cout, P, P, k, k, (s, s), (pad, pad), (1, 1),
                         ksplit=ks)

        go()
        torch.cuda.synchronize()
        if ref is None:
            ref = y.clone()
            err = 0.0
        else:
            err = float((y.float() - ref.float()).abs().max())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            go()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / iters
        res[f"{v}/{ks}"] = (us, err)
        print(f"{name:22s} v{v} ks{ks:2d} {us:8.1f} us  {flops / us / 1e6:7.1f} TF/s  {nbytes / us / 1e3:7.1f} GB/s  maxdiff {err:.3g}",
              flush=True)
    lib().conv_fwd_variant(0)
    return res


def run_wgrad(name, H, Cin, Cout, k, s, N, variants, iters, split_pcts=(100,), slabs=(1,)):
    """dW of the forward conv (Cin -> Cout): the wgrad kernel with M = Cout, N = k*k*Cin."""
    pad = k // 2
    P = (H + 2 * pad - k) // s + 1
    x = torch.randn(N, Cin, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    dy = torch.randn(N, Cout, P, P, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    dw = torch.zeros(Cout * k * k * Cin, device="cuda")
    flops = 2.0 * N * P * P * Cout * Cin * k * k
    ref = None
    res = {}
    for v, sp, sl in [(v, sp, sl) for v in variants for sp in split_pcts for sl in slabs]:
        if True:
            lib().conv_wgrad_tuning(v, sp)
            lib().conv_wgrad_slab(int(sl))

            def go():
                return lib().conv_wgrad(x.data_ptr(), dy.data_ptr(), dw.data_ptr(), N, H, H, Cin, Cin, 1, Cout, P, P,
                                        Cout, k, k, s, s, pad, pad, 1, 1, 0, 0, 0, torch.cuda.current_stream().cuda_stream)

            splits = go()
            torch.cuda.synchronize()
            if ref is None:
                ref = dw.clone()
                err = 0.0
            else:
                err = float(((dw - ref).abs().max() / ref.abs().max().clamp_min(1e-30)))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                go()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / iters
            res[f"{v}/{sp}/{sl}"] = (us, err)
            print(f"wg {name:22s} v{v} split{sp:4d}% ({splits:3d}) { {1: 'slab', 0: 'atom'}.get(sl, 'auto') } {us:8.1f} us  "
                  f"{flops / us / 1e6:7.1f} TF/s  relerr {err:.3g}", flush=True)
    lib().conv_wgrad_tuning(0, 100)
    lib().conv_wgrad_slab(-1)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--variants", default="0,1,2,3,5,7,8,9")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out")
    ap.add_argument("--wgrad", action="store_true")
    ap.add_argument("--splits", default="100")
    ap.add_argument("--slab", default="1", help="wgrad split-K combine: 1 = ordered slabs, 0 = atomics, -1 = heuristic (e.g. 1,0)")
    ap.add_argument("--layers", default="", help="comma-separated layer names (default: all)")
    ap.add_argument("--set", default="resnet50", choices=["resnet50", "hourglass", "yolov3"])
    ap.add_argument("--ksplit", default="1", help="forward split-K factors (e.g. 1,2,3)")
    a = ap.parse_args()
    keep = set(a.layers.split(",")) if a.layers else None
    vs = [int(v) for v in a.variants.split(",")]
    out = {}
    for L in {"hourglass": HOURGLASS, "yolov3": YOLOV3}.get(a.set, LAYERS):
        if keep is not None and L[0] not in keep:
            continue
        if a.wgrad:
            if not L[0].startswith("dg_"):
                out[L[0]] = run_wgrad(*L, a.batch, vs, a.iters, [int(x) for x in a.splits.split(",")],
                                      [int(x) for x in a.slab.split(",")])
        else:
            out[L[0]] = run(*L, a.batch, vs, a.iters, [int(x) for x in a.ksplit.split(",")])
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
