#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/dw_bench.py --variants 0,1,2,3,4,5 > gpurun_out/dw_var.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/dw_var.log | grep -E "H  14|H   7|H  28" | head -80
