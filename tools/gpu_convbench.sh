#!/bin/bash
# conv variant sweeps + GPU tests + bench (one gpurun call)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 300 python tools/bench_conv.py --wgrad --variants 0,1,2,3,4,5,6,7 --splits 50,100,200 --iters 10 --out gpurun_out/wgbench.json > gpurun_out/wgbench.log 2>&1 &&
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
