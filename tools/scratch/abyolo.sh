#!/bin/bash
# same-box YOLOv3 eager: dc76dda tree (ab_old, same kernels) vs the working tree (8 and 4 queues)
mkdir -p gpurun_out/aby; rc=0
for i in 1 2; do
  [ $rc -eq 0 ] && { (cd ab_old && timeout -k 10 240 python bench.py --model yolov3 --steps 20 --warmup 5) > gpurun_out/aby/old_$i.log 2>&1 || rc=$?; }
  [ $rc -eq 0 ] && { timeout -k 10 240 python bench.py --model yolov3 --steps 20 --warmup 5 > gpurun_out/aby/new8_$i.log 2>&1 || rc=$?; }
  [ $rc -eq 0 ] && { DV_KEEP_HW_QUEUES=1 GPU_MAX_HW_QUEUES=4 timeout -k 10 240 python bench.py --model yolov3 --steps 20 --warmup 5 > gpurun_out/aby/new4_$i.log 2>&1 || rc=$?; }
done
for f in gpurun_out/aby/*.log; do echo "$(basename $f .log): $(grep '^{' $f | tail -1 | grep -o '"value": [0-9.]*')"; done
exit $rc
