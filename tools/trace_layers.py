"""Per-layer view of one ResNet-50 training step from a rocprofv3 kernel trace.

usage: python tools/trace_layers.py <run_kernel_trace.csv> [step index from the end, default 1]
Splits the trace into steps at the SGD kernel, then lists every kernel of the chosen step in
dispatch order with its duration, grid and the gap to the previous kernel's end (launch /
dependency bubbles), plus totals of kernel time vs. wall time of the step.
"""
import csv
import re
import sys


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"\(.*", "", n)
    return n[:60]


def main():
    rows = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Grid_Size_X"]),
                         int(r["Workgroup_Size_X"])))
    rows.sort()
    which = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    ends = [i for i, r in enumerate(rows) if re.search(r"(sgd|adam|rmsprop)_kernel", r[2])]
    if len(ends) < which + 1:
        sys.exit("not enough steps in the trace")
    a, b = ends[-which - 1] + 1, ends[-which] + 1
    step = rows[a:b]
    t0 = step[0][0]
    prev_end = step[0][0]
    busy = 0
    gaps = 0
    for s, e, n, g, wg in step:
        gap = max(0, s - prev_end)
        gaps += gap
        busy += e - s
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} us  gap {gap / 1e3:6.1f}  blocks {g // max(wg, 1):7d}  {short(n)}")
        prev_end = max(prev_end, e)
    wall = step[-1][1] - step[0][0]
    print(f"\nkernels {len(step)}  busy {busy / 1e6:.3f} ms  gaps {gaps / 1e6:.3f} ms  wall {wall / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
