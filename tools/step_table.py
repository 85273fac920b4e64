"""Per-step kernel table from a rocprofv3 kernel trace: only the steady-state steps (dispatches
between consecutive optimizer kernels, the last ``--steps`` of them) are counted, so one-time
setup (weight-cache builds, parameter copies, first-step fills) does not leak into the per-step
numbers the way a whole-run ``--stats`` average does.

python tools/step_table.py <run_kernel_trace.csv> [--steps 3] [--title ...] [--marker REGEX]
"""
import argparse
import csv
import re
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import family  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--title", default="")
    ap.add_argument("--marker", default="(sgd|adam|rmsprop)_kernel")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if re.search(a.marker, r["Kernel_Name"])]
    k = min(a.steps, len(idx) - 1)
    if k < 1:
        raise SystemExit("fewer than two optimizer dispatches in the trace")
    lo, hi = idx[-k - 1], idx[-1]
    stats = {}
    busy = 0.0
    for r in rows[lo + 1: hi + 1]:
        n = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        s = stats.setdefault(n, [0, 0.0])
        s[0] += 1
        s[1] += d
        busy += d
    span = (int(rows[hi]["End_Timestamp"]) - int(rows[lo]["End_Timestamp"])) / 1e3
    total = busy / k / 1e3
    print(f"# {a.title}")
    print(f"# steady state: the last {k} steps of the trace ({(hi - lo) / k:.0f} dispatches per step)")
    print(f"# kernel time per step: {total:.3f} ms; step span (first to last dispatch end): {span / k / 1e3:.3f} ms")
    fam = {}
    for n, (c, t) in stats.items():
        fam[family(n)] = fam.get(family(n), 0.0) + t / k / 1e3
    print("\n# by family (ms/step)")
    for f, v in sorted(fam.items(), key=lambda kv: -kv[1]):
        print(f"  {v:7.3f}  {100 * v / total:5.1f}%  {f}")
    print("\n ms/step calls/step   avg_us  kernel")
    for n, (c, t) in sorted(stats.items(), key=lambda kv: -kv[1][1]):
        print(f"  {t / k / 1e3:7.3f}  {c / k:9.1f}  {t / c:7.1f}  {n[:150]}")


if __name__ == "__main__":
    main()
