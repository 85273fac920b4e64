"""Loss-curve sweep: native HIP path vs PyTorch autocast-bf16 from identical initial weights.

usage: python tools/lc_sweep.py [--models resnet50,mobilenet1] [--seeds 0,1,2] [--steps 100] [--batch 64]
                                [--grid 0.05:1.0,0.02:1.0,0.02:0.3,0.01:0.3] [--out profiles/loss_curve_sweep.txt]

Each (model, lr, noise, seed) trains the learnable 16-class task of tools/loss_curve.py with
SGD(m=0.9, wd=1e-4). High-lr runs are chaotic (single-seed finals swing by orders of magnitude
between two bf16 roundings of the same model), so the comparison is the median final loss over
seeds per arm, plus the per-seed finals.
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from loss_curve import run_curve  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="resnet50,mobilenet1")
    ap.add_argument("--seeds", default="0,1,2")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--grid", default="0.05:1.0,0.02:1.0,0.02:0.3,0.01:0.3")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    seeds = [int(s) for s in a.seeds.split(",")]
    lines = [f"# tools/lc_sweep.py: batch {a.batch}, {a.steps} SGD(m=0.9, wd=1e-4) steps, learnable 16-class task; "
             f"seeds {a.seeds}; columns: model lr noise arm median-final | per-seed finals | seed-0 loss[::10]"]
    for name in a.models.split(","):
        for cell in a.grid.split(","):
            lr, noise = (float(v) for v in cell.split(":"))
            finals, first = {}, {}
            for sd in seeds:
                c = run_curve(name, bs=a.batch, steps=a.steps, lr=lr, noise=noise, seed=sd)
                for arm, ls in c.items():
                    finals.setdefault(arm, []).append(ls[-1])
                    first.setdefault(arm, ls[::10])
            for arm, fs in finals.items():
                ln = f"{name} {lr} {noise} {arm} {statistics.median(fs):.4f} | {fs} | {first[arm]}"
                print(ln, flush=True)
                lines.append(ln)
    if a.out:
        with open(a.out, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
