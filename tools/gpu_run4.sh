set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_ops_gpu.py -q -m gpu > gpurun_out/t4.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench4.log 2>&1 && \
timeout -k 10 500 python bench/conv_bench.py --iters 10 --json gpurun_out/conv_bench4.json > gpurun_out/conv_bench4.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof4 -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/prof4.log 2>&1
