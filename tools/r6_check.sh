#!/bin/bash
# round-6 check: GPU tests, 1-GPU ResNet-50 bench (+ single-stream A/B), input pipeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 900 $PYT tests -m gpu > gpurun_out/tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --model yolov3 --steps 10 --warmup 3 > gpurun_out/bench_yolo.log 2>&1 && \
timeout -k 10 300 python bench.py --model hourglass --steps 10 --warmup 3 > gpurun_out/bench_hg.log 2>&1 && \
timeout -k 10 600 python -u bench/input_pipeline.py --images 1536 --per-worker 256 --workers 1,4,8,16 --batch 128 --batches 24 --out gpurun_out/input_pipeline_shm.json > gpurun_out/input_pipeline_shm.log 2>&1
rc=$?
tail -3 gpurun_out/tests.log; grep -E "^FAILED" gpurun_out/tests.log | head
for f in bench bench_yolo bench_hg; do tail -1 gpurun_out/$f.log | cut -c1-260; done
tail -2 gpurun_out/input_pipeline_shm.log | cut -c1-600
exit $rc
