#!/bin/bash
# BN-deferral check on one GPU: the bitwise A/B tests, then the ResNet-50 bench with the deferral
# on and off, then (PROF=1) rocprof kernel tables of both arms (tools/prof_ab.sh).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_defer_gpu.py > gpurun_out/defer_tests.log 2>&1
rc=$?; tail -6 gpurun_out/defer_tests.log
if [ $rc -eq 0 ]; then
  DV_DEFER=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_defer.log 2>&1 && \
  DV_DEFER=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_nodefer.log 2>&1
  rc=$?
  tail -1 gpurun_out/bench_defer.log | cut -c1-200; tail -1 gpurun_out/bench_nodefer.log | cut -c1-200
fi
if [ $rc -eq 0 ] && [ -n "$PROF" ]; then bash tools/prof_ab.sh > /dev/null 2>&1; rc=$?; fi
exit $rc
