"""Per-kernel timeline of one training step from a rocprofv3 kernel trace.

python tools/trace_step.py <run_kernel_trace.csv> [--marker sgd_kernel] [--which -1]
Prints every dispatch between two optimizer kernels with duration, idle gap before the next
dispatch, grid and VGPR/LDS usage, then the busy/idle totals.
"""
import argparse
import csv
import re


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    n = re.sub(r"\(.*$", "", n) if not n.startswith("at::") else n[:60]
    return n[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--marker", default="(sgd|adam|rmsprop)_kernel", help="regex of the step-ending kernel")
    ap.add_argument("--which", type=int, default=-1)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if re.search(a.marker, r["Kernel_Name"])]
    lo, hi = idx[a.which - 1], idx[a.which]
    busy = idle = 0.0
    for i in range(lo + 1, hi + 1):
        r = rows[i]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        g = (int(rows[i + 1]["Start_Timestamp"]) - int(r["End_Timestamp"])) / 1e3 if i + 1 < len(rows) else 0.0
        busy += d
        idle += max(g, 0.0) if i < hi else 0.0
        grid = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        print(f"{i - lo:4d} {d:8.1f}us idle {g:7.1f}  blocks {grid:7d} vgpr {r['VGPR_Count']:>3} lds {r['LDS_Block_Size']:>6}  {short(r['Kernel_Name'])}")
    span = (int(rows[hi]["End_Timestamp"]) - int(rows[lo]["End_Timestamp"])) / 1e3
    print(f"step span {span / 1e3:.3f} ms  busy {busy / 1e3:.3f} ms  idle {idle / 1e3:.3f} ms  dispatches {hi - lo}")


if __name__ == "__main__":
    main()
