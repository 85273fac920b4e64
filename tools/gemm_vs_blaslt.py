"""1x1 stride-1 convs of ResNet-50 are plain GEMMs in NHWC: time the native kernels against
hipBLASLt (torch.mm, bf16) on the same shapes, interleaved in one process.

  fwd   Y[M,N]  = X[M,K] W[N,K]^T      (native: conv_fwd, plain and with the BN-stats epilogue)
  dgrad dX[M,K] = dY[M,N] W[N,K]
  wgrad dW[N,K] = dY[M,N]^T X[M,K]      (native: conv_wgrad, split-K, fp32 out)

python tools/gemm_vs_blaslt.py [--batch 256] [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from deep_vision_amd._ext import lib  # noqa: E402
from deep_vision_amd.ops.bn import STAT_ROWS  # noqa: E402
from deep_vision_amd.ops.conv import conv_fwd_raw  # noqa: E402

# (Cin, Cout, H, count)
SHAPES = [(64, 64, 56, 1), (64, 256, 56, 4), (256, 64, 56, 2), (128, 512, 28, 4), (512, 128, 28, 3),
          (256, 1024, 14, 6), (1024, 256, 14, 5), (512, 2048, 7, 3), (2048, 512, 7, 2)]


def timeit(fn, iters):
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
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    N = a.batch
    st = torch.cuda.current_stream().cuda_stream
    tot = {}
    print(f"{'layer':16s} {'pass':6s} {'native':>9s} {'native+st':>9s} {'blaslt':>9s}  {'memGB/s(n)':>10s}")
    for Cin, Cout, H, cnt in SHAPES:
        M = N * H * H
        x = torch.randn(M, Cin, device="cuda").bfloat16()
        w = (torch.randn(Cout, Cin, device="cuda") * 0.05).bfloat16()
        dy = torch.randn(M, Cout, device="cuda").bfloat16()
        y = torch.empty(M, Cout, device="cuda", dtype=torch.bfloat16)
        dx = torch.empty(M, Cin, device="cuda", dtype=torch.bfloat16)
        wt = w.t().contiguous()
        stats = torch.zeros(STAT_ROWS, Cout, device="cuda")  # shard sums + shift row (csrc/kernels.h)
        dw = torch.zeros(Cout, Cin, device="cuda")

        def f_nat():
            conv_fwd_raw(x, w, y, None, None, N, H, H, Cin, Cin, 1, Cout, H, H, 1, 1, (1, 1), (0, 0), (1, 1))

        def f_nat_st():
            conv_fwd_raw(x, w, y, None, stats, N, H, H, Cin, Cin, 1, Cout, H, H, 1, 1, (1, 1), (0, 0), (1, 1))

        def f_bl():
            torch.mm(x, wt, out=y)

        def d_nat():  # weight operand for dgrad: [Cin][Cout]
            conv_fwd_raw(dy, wt, dx, None, None, N, H, H, Cout, Cout, 1, Cin, H, H, 1, 1, (1, 1), (0, 0), (1, 1))

        def d_bl():
            torch.mm(dy, w, out=dx)

        def g_nat():
            lib().conv_wgrad(x.data_ptr(), dy.data_ptr(), dw.data_ptr(), N, H, H, Cin, Cin, 1, Cout, H, H, Cout, 1, 1,
                             1, 1, 0, 0, 1, 1, 0, 0, 0, st)

        def g_bl():
            torch.mm(dy.t(), x, out=dwb)

        dwb = torch.empty(Cout, Cin, device="cuda", dtype=torch.bfloat16)
        name = f"{Cin}->{Cout}@{H}"
        byts = 2.0 * M * (Cin + Cout)
        for pas, fns in (("fwd", (f_nat, f_nat_st, f_bl)), ("dgrad", (d_nat, None, d_bl)), ("wgrad", (g_nat, None, g_bl))):
            ts = []
            for rnd in range(2):  # interleaved rounds, keep the min
                ts.append([timeit(f, a.iters) if f is not None else float("nan") for f in fns])
            t = [min(r[i] for r in ts) for i in range(3)]
            for i, k in enumerate(("nat", "nat_st", "bl")):
                if t[i] == t[i]:
                    tot[(pas, k)] = tot.get((pas, k), 0.0) + t[i] * cnt
            print(f"{name:16s} {pas:6s} {t[0]:9.1f} {t[1]:9.1f} {t[2]:9.1f}  {byts / t[0] / 1e3:10.0f}", flush=True)
    print("weighted per-step totals (us):")
    for k, v in sorted(tot.items()):
        print(f"  {k[0]:6s} {k[1]:7s} {v:9.1f}")


if __name__ == "__main__":
    main()
