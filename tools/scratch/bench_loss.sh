#!/bin/bash
mkdir -p gpurun_out/bl; rc=0
for spec in "resnet50" "mobilenet1 --graph" "inception1"; do
  set -- $spec; m=$1; shift
  [ $rc -eq 0 ] && { timeout -k 10 240 python bench.py --model $m "$@" --steps 20 --warmup 5 > gpurun_out/bl/$m.log 2>&1 || rc=$?; }
  echo "$m $*: $(grep '^{' gpurun_out/bl/$m.log | tail -1 | grep -o '"value": [0-9.]*\|"loss_first_last": \[[^]]*\]' | tr '\n' ' ')"
done
exit $rc
