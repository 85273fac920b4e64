#!/bin/bash
mkdir -p gpurun_out/abc; rc=0
for i in 1 2; do for m in side flush; do
  [ $rc -eq 0 ] && { DV_WGRAD_SIDE_COMM=$m timeout -k 10 240 python bench.py --force-dp --steps 30 --warmup 5 > gpurun_out/abc/${m}_$i.log 2>&1 || rc=$?; }
  echo "resnet50 force-dp comm=$m run $i: $(grep '^{' gpurun_out/abc/${m}_$i.log | tail -1 | grep -o '"value": [0-9.]*')"
done; done
exit $rc
