"""ResNet-50 stem conv (7x7 s2, 3 -> 64, batch 256 @ 224, bf16) forward and weight gradient:
dedicated row-walking kernels (csrc/stem.hip) vs the packed implicit-GEMM path vs PyTorch/MIOpen.
Times are per call (HIP events over 10 calls after 3 warm-up calls); the native forward includes
the tap-pack pass, the weight gradient includes its reduce pass.
usage: python tools/stem_bench.py [--blocks 256,512,1024] [--batch 256]"""
import argparse
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from deep_vision_amd import ops as F  # noqa: E402
from deep_vision_amd._ext import lib  # noqa: E402
from deep_vision_amd.ops import conv as C  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", default="512:256", help="fwd:wgrad target grids, comma-separated")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--native-only", action="store_true", help="skip the generic-path and MIOpen arms (profiling)")
    a = ap.parse_args()
    torch.manual_seed(0)
    x = torch.randn(a.batch, 3, 224, 224, device="cuda")
    w = (torch.randn(64, 3, 7, 7, device="cuda") * 0.05).requires_grad_(True)
    flop = 2 * a.batch * 112 * 112 * 64 * 147
    y = F.conv2d(x, w, None, 2, 3)
    g = torch.randn(y.shape, device="cuda").bfloat16().to(memory_format=torch.channels_last)  # as autograd hands it over

    def fwd():
        F.conv2d(x, w, None, 2, 3)

    def wgrad():
        yy = F.conv2d(x, w, None, 2, 3)
        torch.autograd.grad(yy, w, g)

    rows = []
    for mode in ([] if a.native_only else ["generic"]) + [f"stem:{b}" for b in a.blocks.split(",")]:
        C.STEM_KERNELS = mode != "generic"
        if mode != "generic":
            lib().stem_tuning(int(mode.split(":")[1]), int(mode.split(":")[2]))
        f = timeit(fwd)
        fb = timeit(wgrad)
        rows.append((mode, f, fb - f))
    C.STEM_KERNELS = True
    lib().stem_tuning(0, 0)
    if a.native_only:
        for m, f, wg in rows:
            print(f"{m:12s} fwd {f:7.1f} us   wgrad {wg:7.1f} us")
        return
    # PyTorch / MIOpen reference (bf16 NHWC, same shapes)
    xt = x.bfloat16().contiguous(memory_format=torch.channels_last)
    wt = w.detach().bfloat16().contiguous(memory_format=torch.channels_last).requires_grad_(True)
    gt = g
    conv = torch.nn.functional.conv2d
    f = timeit(lambda: conv(xt, wt, None, 2, 3))
    fb = timeit(lambda: torch.autograd.grad(conv(xt, wt, None, 2, 3), wt, gt))
    rows.append(("miopen", f, fb - f))
    print(f"# tools/stem_bench.py: ResNet-50 stem 7x7/2 3->64, batch {a.batch} @224, bf16, 1x MI355X")
    for m, f, wg in rows:
        print(f"{m:12s} fwd {f:7.1f} us ({flop / f / 1e6:6.1f} TF)   wgrad {wg:7.1f} us ({flop / wg / 1e6:6.1f} TF)",
              flush=True)
    # numerics: dedicated vs generic on the same inputs
    C.STEM_KERNELS = True
    y1 = F.conv2d(x, w, None, 2, 3).float()
    d1 = torch.autograd.grad(F.conv2d(x, w, None, 2, 3), w, g)[0].detach()
    C.STEM_KERNELS = False
    y0 = F.conv2d(x, w, None, 2, 3).float()
    d0 = torch.autograd.grad(F.conv2d(x, w, None, 2, 3), w, g)[0].detach()
    C.STEM_KERNELS = True
    print(f"# max|y diff| {float((y1 - y0).abs().max()):.3e}  rel dW diff {float((d1 - d0).norm() / d0.norm()) if d0.norm() > 0 else 0.0:.3e}")


if __name__ == "__main__":
    main()
