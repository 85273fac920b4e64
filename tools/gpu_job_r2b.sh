#!/bin/bash
# GPU tests, then depthwise variant bench and model benches (each step time-limited, chained).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread ${TESTS:-tests} -m gpu > gpurun_out/tests.log 2>&1
rc=$?; tail -3 gpurun_out/tests.log; grep -E "^FAILED" gpurun_out/tests.log | head
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/dw_bench.py --variants 0,9 --iters 10 > gpurun_out/dw.log 2>&1 || exit $?
for m in ${MODELS:-mobilenet1 hourglass resnet50}; do
  timeout -k 10 300 python bench.py --model $m --steps 10 --warmup 3 > gpurun_out/bench_$m.log 2>&1 || exit $?
  echo "$m: $(tail -1 gpurun_out/bench_$m.log | cut -c1-200)"
done
