#!/bin/bash
mkdir -p gpurun_out
bad() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py tests/test_heads_gpu.py \
  tests/test_graph_gpu.py tests/test_branch_streams_gpu.py > gpurun_out/t_b.log 2>&1
rc=$?; tail -2 gpurun_out/t_b.log; grep -E "^FAILED|^E  " gpurun_out/t_b.log | head -20
bad $rc && exit $rc
for m in hourglass yolov3 resnet50 mobilenet1; do
  timeout -k 10 300 python bench.py --model $m --steps 10 --warmup 3 > gpurun_out/b_$m.log 2>&1 || exit $?
  echo "$m eager $(tail -1 gpurun_out/b_$m.log | cut -c60-130)"
done
timeout -k 10 300 python -u tools/host_profile.py --model hourglass --steps 3 --top 5 > gpurun_out/host_hourglass.log 2>&1 || exit $?
sed -n 1,14p gpurun_out/host_hourglass.log | grep -v amdgpu | cut -c1-150
