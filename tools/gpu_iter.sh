# one build->measure iteration: microbenches, full GPU tests, bench, profile
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_heads_gpu.py -x -q -k "fused_in_dgrad or grad_join" --timeout 120 --timeout-method thread > gpurun_out/t_first.log 2>&1 && \
timeout -k 10 300 python tools/bn_bench.py --rounds 2 > gpurun_out/bn_bench.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r50 -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/prof_r50.log 2>&1
rc=$?
cd $R
tail -3 gpurun_out/t_first.log; grep "blocks= 1024 unroll=2" gpurun_out/bn_bench.log; tail -2 gpurun_out/tests.log; tail -1 gpurun_out/bench.log | cut -c1-200
echo rc=$rc
exit $rc
