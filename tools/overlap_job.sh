#!/bin/bash
# Bucket all-reduce overlap evidence on one GPU (world-1 RCCL, DataParallel forced on): the
# issue-order GPU test, then a rocprofv3 kernel trace of the force-DP ResNet-50 step summarised
# by tools/comm_timeline.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_ddp_gpu.py -k overlap \
  > gpurun_out/overlap_test.log 2>&1
rc=$?; grep -E "PASS|FAIL|backward .* ms" gpurun_out/overlap_test.log | head
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/gpurun_out/prof_dp" -o run --output-format csv -- \
  python3 "$R/bench.py" --force-dp --bucket-mb 8 --steps 3 --warmup 2 > "$R/gpurun_out/prof_dp.log" 2>&1
rc=$?; cd "$R"
t=$(find gpurun_out/prof_dp -name '*kernel_trace.csv' -print -quit)
[ -n "$t" ] && python tools/comm_timeline.py "$t" > gpurun_out/comm_timeline.txt 2>&1; rm -f "$t"
head -40 gpurun_out/comm_timeline.txt
exit $rc
