#!/bin/bash
# host-side (Python) profiles of the eager launch-bound models + their eager bench numbers
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python tools/host_profile.py --model hourglass --steps 5 --top 45 > gpurun_out/host_hourglass.txt 2>&1 && \
timeout -k 10 300 python tools/host_profile.py --model yolov3 --steps 5 --top 45 > gpurun_out/host_yolov3.txt 2>&1 && \
timeout -k 10 300 python bench.py --model hourglass --steps 10 --warmup 3 > gpurun_out/host_bench_hg.log 2>&1
rc=$?
head -30 gpurun_out/host_hourglass.txt | cut -c1-150; grep '^{' gpurun_out/host_bench_hg.log | cut -c1-120
exit $rc
