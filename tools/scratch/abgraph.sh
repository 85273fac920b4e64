#!/bin/bash
# same-box A/B under 8 HW queues: weight-gradient side stream off (0) / on (1) in captured steps
mkdir -p gpurun_out/abg; rc=0
for spec in "yolov3 --graph" "resnet50 --graph" ; do
  set -- $spec; m=$1; shift; a="$*"
  for i in 1 2; do for s in 0 1; do
    [ $rc -eq 0 ] || break
    DV_WGRAD_SIDE=$s timeout -k 10 240 python bench.py --model $m $a --steps 20 --warmup 5 > gpurun_out/abg/${m}_${s}_$i.log 2>&1 || rc=$?
    echo "$m $a SIDE=$s run $i: $(grep '^{' gpurun_out/abg/${m}_${s}_$i.log | tail -1 | cut -c60-110)"
  done; done
done
for s in 0 1; do
  [ $rc -eq 0 ] || break
  DV_KEEP_HW_QUEUES=1 GPU_MAX_HW_QUEUES=4 DV_WGRAD_SIDE=$s timeout -k 10 240 python bench.py --model resnet50 --graph --steps 20 --warmup 5 > gpurun_out/abg/q4_${s}.log 2>&1 || rc=$?
  echo "resnet50 --graph 4 queues SIDE=$s: $(grep '^{' gpurun_out/abg/q4_${s}.log | tail -1 | cut -c60-110)"
done
exit $rc
