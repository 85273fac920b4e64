#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -s --timeout 200 --timeout-method thread tests/test_branch_streams_gpu.py > gpurun_out/t_b.log 2>&1
rc=$?; tail -2 gpurun_out/t_b.log; grep -E "^FAILED|^E  " gpurun_out/t_b.log | head -20; exit $rc
