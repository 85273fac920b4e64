"""Launch census of one training step (rocprofv3 kernel trace): per kernel family, how many
launches the step issues and their total / median duration -- the view for launch-bound models
(Stacked Hourglass, YOLOv3), where the count matters as much as the time.

usage: python tools/kernel_census.py <run_kernel_trace.csv>
"""
import collections
import csv
import re
import statistics
import sys


def family(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    n = re.sub(r"\(.*$", "", n)
    if n.startswith("at::"):
        n = "torch:" + re.sub(r"<.*", "", n.split("::")[-1])[:30]
    return re.sub(r"<.*", "", n)


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if re.search(r"(sgd|adam|rmsprop)_kernel", r["Kernel_Name"])]
    lo, hi = idx[-2], idx[-1]
    step = rows[lo + 1:hi + 1]
    by = collections.defaultdict(list)
    for r in step:
        by[family(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    span = (int(step[-1]["End_Timestamp"]) - int(rows[lo]["End_Timestamp"])) / 1e3
    busy = sum(sum(v) for v in by.values())
    print(f"step: {len(step)} launches, busy {busy / 1e3:.3f} ms, span {span / 1e3:.3f} ms")
    print(f"{'launches':>8} {'total_ms':>9} {'median_us':>9}  kernel")
    for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        print(f"{len(v):8d} {sum(v) / 1e3:9.3f} {statistics.median(v):9.1f}  {k}")


if __name__ == "__main__":
    main()
