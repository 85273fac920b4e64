#!/bin/bash
# rocprofv3 kernel stats of the ResNet-50 bench step with the BN deferral off and on (A/B).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
rc=0
for d in 0 1; do
  DV_DEFER=$d timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_defer$d" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 > "$R/gpurun_out/prof_defer$d.log" 2>&1 || { rc=$?; break; }
done
cd "$R"
for d in 0 1; do
  f=$(find gpurun_out/prof_defer$d -name '*kernel_stats.csv' -print -quit)
  [ -n "$f" ] && python tools/prof_summary.py "$f" 7 "resnet50 DV_DEFER=$d bench.py --steps 5 --warmup 2" > gpurun_out/prof_defer$d.txt 2>&1
  t=$(find gpurun_out/prof_defer$d -name '*kernel_trace.csv' -print -quit)
  [ -n "$t" ] && python tools/trace_layers.py "$t" > gpurun_out/layers_defer$d.txt 2>&1; rm -f "$t"
done
head -45 gpurun_out/prof_defer0.txt | cut -c1-150; head -45 gpurun_out/prof_defer1.txt | cut -c1-150
exit $rc
