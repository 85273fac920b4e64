set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q -k "depthwise" --timeout 120 --timeout-method thread > gpurun_out/t_dw.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_heads_gpu.py -x -q -k "classifiers" --timeout 200 --timeout-method thread > gpurun_out/t_cls.log 2>&1 && \
timeout -k 10 300 python bench.py --model mobilenet1 --steps 10 --warmup 3 > gpurun_out/bench_mobilenet1.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_mb -o run --output-format csv -- python3 $R/bench.py --model mobilenet1 --steps 5 --warmup 2 > $R/gpurun_out/prof_mb.log 2>&1
rc=$?
cd $R
tail -2 gpurun_out/t_dw.log; tail -2 gpurun_out/t_cls.log; tail -1 gpurun_out/bench_mobilenet1.log | cut -c1-180
echo rc=$rc
exit $rc
