#!/bin/bash
mkdir -p gpurun_out
for v in 0 25165824 0 25165824 999999999999; do
DV_NT_MIN=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b_resnet50.log 2>&1 || exit $?
echo "NT_MIN=$v $(tail -1 gpurun_out/b_resnet50.log | cut -c80-120)"
done
