#!/bin/bash
mkdir -p gpurun_out/abq16; rc=0
for i in 1 2; do for q in 8 16; do
  [ $rc -eq 0 ] && { GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python bench.py --steps 30 --warmup 5 > gpurun_out/abq16/r_${q}_$i.log 2>&1 || rc=$?; }
  echo "resnet50 eager queues=$q run $i: $(grep '^{' gpurun_out/abq16/r_${q}_$i.log | tail -1 | grep -o '"value": [0-9.]*')"
done; done
exit $rc
