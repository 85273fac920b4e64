#!/bin/bash
# GPU tests for the current changes + convergence pilot + benches; stops at the first crash / timeout
mkdir -p gpurun_out
bad() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 900 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_branch_streams_gpu.py \
  tests/test_ops_gpu.py tests/test_bn_numerics_gpu.py tests/test_heads_gpu.py tests/test_graph_gpu.py \
  tests/test_prodshape_gpu.py > gpurun_out/t_b.log 2>&1
rc=$?; tail -3 gpurun_out/t_b.log; grep -E "run-to-run|^FAILED|^E " gpurun_out/t_b.log | head -20
bad $rc && exit $rc
for m in resnet50; do
  timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/b_$m.log 2>&1 || exit $?
  tail -1 gpurun_out/b_$m.log | cut -c1-200
done
for m in hourglass yolov3; do
  timeout -k 10 300 python bench.py --model $m --steps 10 --warmup 3 --graph > gpurun_out/bg_$m.log 2>&1 || exit $?
  tail -1 gpurun_out/bg_$m.log | cut -c1-200
done
timeout -k 10 500 python -u tools/convergence.py --steps 300 --seeds 0 --every 50 > gpurun_out/conv_pilot.log 2>&1
rc=$?; tail -20 gpurun_out/conv_pilot.log; bad $rc && exit $rc
timeout -k 10 300 python -u tools/host_profile.py --model hourglass --steps 3 > gpurun_out/host_hg.log 2>&1 || exit $?
head -60 gpurun_out/host_hg.log | cut -c1-160
