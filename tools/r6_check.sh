#!/bin/bash
# round-6 check: GPU tests, smoke, 1-GPU benches of the BASELINE models
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 900 $PYT tests -m gpu > gpurun_out/tests.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --model yolov3 --steps 20 --warmup 5 > gpurun_out/bench_yolo.log 2>&1 && \
timeout -k 10 300 python bench.py --model hourglass --steps 20 --warmup 5 > gpurun_out/bench_hg.log 2>&1 && \
timeout -k 10 300 python bench.py --model mobilenet1 --steps 20 --warmup 5 > gpurun_out/bench_mob.log 2>&1
rc=$?
tail -3 gpurun_out/tests.log; grep -E "^FAILED" gpurun_out/tests.log | head
tail -2 gpurun_out/smoke.log
for f in bench bench_yolo bench_hg bench_mob; do tail -1 gpurun_out/$f.log | cut -c1-230; done
exit $rc
