#!/bin/bash
mkdir -p gpurun_out
for v in "DV_NT_MIN=0" "DV_NT_MIN=25165824" "DV_EPI_NT_MIN=999999999999" "DV_NT_MIN=0" "DV_NT_MIN=25165824" "DV_EPI_NT_MIN=999999999999"; do
env $v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b_resnet50.log 2>&1 || exit $?
echo "$v $(tail -1 gpurun_out/b_resnet50.log | cut -c80-120)"
done
