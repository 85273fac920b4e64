#!/bin/bash
mkdir -p gpurun_out
bad() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k conv > gpurun_out/t_b.log 2>&1
rc=$?; tail -1 gpurun_out/t_b.log; bad $rc && exit $rc
for v in 25165824 999999999999 25165824 999999999999; do
DV_XNT_MIN=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b_resnet50.log 2>&1 || exit $?
echo "XNT=$v $(tail -1 gpurun_out/b_resnet50.log | cut -c80-120)"
done
