#!/bin/bash
mkdir -p gpurun_out
bad() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 900 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_branch_streams_gpu.py \
  tests/test_ops_gpu.py tests/test_bn_numerics_gpu.py tests/test_heads_gpu.py tests/test_graph_gpu.py \
  tests/test_prodshape_gpu.py tests/test_defer_gpu.py tests/test_ddp_gpu.py > gpurun_out/t_b.log 2>&1
rc=$?; tail -3 gpurun_out/t_b.log; grep -E "^FAILED|^E  " gpurun_out/t_b.log | head -20
bad $rc && exit $rc
timeout -k 10 300 python bench.py --model hourglass --steps 10 --warmup 3 --graph > gpurun_out/bg_hourglass.log 2>&1 || exit $?
tail -1 gpurun_out/bg_hourglass.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b_resnet50.log 2>&1 || exit $?
tail -1 gpurun_out/b_resnet50.log | cut -c1-200
