set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_ops_gpu.py -q -m gpu > gpurun_out/t3.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench3.log 2>&1 && \
timeout -k 10 500 python bench/conv_bench.py --iters 10 --only fwd --json gpurun_out/conv_bench3.json > gpurun_out/conv_bench3.log 2>&1
