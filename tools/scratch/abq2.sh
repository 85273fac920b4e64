#!/bin/bash
# same-box: captured steps (side stream off in capture) under 8 vs 4 HW queues
mkdir -p gpurun_out/abq2; rc=0
for m in resnet50 yolov3 hourglass mobilenet1; do
  for i in 1 2; do for q in 8 4; do
    [ $rc -eq 0 ] || break
    DV_KEEP_HW_QUEUES=1 GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python bench.py --model $m --graph --steps 20 --warmup 5 > gpurun_out/abq2/${m}_${q}_$i.log 2>&1 || rc=$?
    echo "$m --graph queues=$q run $i: $(grep '^{' gpurun_out/abq2/${m}_${q}_$i.log | tail -1 | grep -o '"value": [0-9.]*')"
  done; done
done
for q in 8 4; do
  [ $rc -eq 0 ] || break
  DV_KEEP_HW_QUEUES=1 GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python bench.py --model yolov3 --steps 20 --warmup 5 > gpurun_out/abq2/yolo_eager_${q}.log 2>&1 || rc=$?
  echo "yolov3 eager queues=$q: $(grep '^{' gpurun_out/abq2/yolo_eager_${q}.log | tail -1 | grep -o '"value": [0-9.]*')"
done
exit $rc
