#!/bin/bash
mkdir -p gpurun_out
bad() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py -k "conv or darknet" > gpurun_out/t_b.log 2>&1
rc=$?; tail -2 gpurun_out/t_b.log; grep -E "^FAILED|^E  " gpurun_out/t_b.log | head -20
bad $rc && exit $rc
for v in 1 0 1 0; do
  DV_WG_FINAL=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b_resnet50.log 2>&1 || exit $?
  echo "FINAL=$v $(tail -1 gpurun_out/b_resnet50.log | cut -c80-140)"
  DV_WG_FINAL=$v timeout -k 10 300 python bench.py --model yolov3 --steps 10 --warmup 3 --graph > gpurun_out/bg_yolov3.log 2>&1 || exit $?
  echo "FINAL=$v $(tail -1 gpurun_out/bg_yolov3.log | cut -c60-120)"
done
