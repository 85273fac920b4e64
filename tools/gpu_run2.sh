set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_ops_gpu.py -q -m gpu > gpurun_out/t2.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench2.log 2>&1 && \
timeout -k 10 500 python bench/conv_bench.py --iters 10 --json gpurun_out/conv_bench.json > gpurun_out/conv_bench.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1; \
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS -d $R/gpurun_out/pmc1 -o c --output-format csv -- python3 $R/tools/conv_one.py 64 64 56 3 1 1 fwd > $R/gpurun_out/pmc1.log 2>&1
