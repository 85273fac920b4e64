"""Summarise a rocprofv3 --kernel-trace --stats run into per-step kernel times.

usage: python tools/prof_summary.py <run_kernel_stats.csv> <dispatch rounds> [title] [bench.log]
       rounds = warmup + steps of the profiled bench.py run (the stats cover every dispatch).
Groups kernels into families (conv fwd/dgrad, wgrad, BN fwd, BN bwd, pool, optimizer, other).
"""
import csv
import json
import re
import sys


def family(name):
    n = name
    if "conv_fwd_kernel" in n:
        return "conv fwd+dgrad (MFMA implicit GEMM)"
    if "conv_wgrad_kernel" in n:
        return "conv wgrad (MFMA split-K)"
    if "bn_bwd" in n:
        return "BN backward"
    if "bn_" in n:
        return "BN forward"
    if "pool" in n or "gap_" in n or "upsample" in n:
        return "pooling"
    if "sgd" in n or "adam" in n or "rmsprop" in n or "wprep" in n or "unprep" in n:
        return "optimizer + weight prep"
    if "dw_" in n:
        return "depthwise conv"
    return "other"


def main():
    path, rounds = sys.argv[1], int(sys.argv[2])
    title = sys.argv[3] if len(sys.argv) > 3 else path
    bench = None
    if len(sys.argv) > 4:
        for line in open(sys.argv[4]):
            if line.startswith("{"):
                bench = json.loads(line)
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e3))
    rows.sort(key=lambda r: -r[2])
    total = sum(r[2] for r in rows) / rounds
    fam = {}
    for n, c, t, a in rows:
        fam[family(n)] = fam.get(family(n), 0.0) + t / rounds
    print(f"# {title}")
    print(f"# per-step = total / {rounds} dispatch rounds (includes one-time setup kernels)")
    line = f"# total kernel time per step: {total:.3f} ms"
    if bench:
        line += f"; bench: {bench['value']:.0f} img/s ({bench['ms_per_step']:.2f} ms/step)"
    print(line)
    print("\n# by family (ms/step)")
    for k, v in sorted(fam.items(), key=lambda kv: -kv[1]):
        print(f"  {v:7.3f}  {100 * v / total:5.1f}%  {k}")
    print("\n ms/step calls/step   avg_us  kernel")
    for n, c, t, a in rows:
        short = re.sub(r"\(anonymous namespace\)::", "", n)
        print(f"{t / rounds:8.3f} {c / rounds:10.1f} {a:8.1f}  {short[:150]}")


if __name__ == "__main__":
    main()
