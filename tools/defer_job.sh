set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_defer_gpu.py > gpurun_out/defer_tests.log 2>&1
rc=$?; tail -15 gpurun_out/defer_tests.log
if [ $rc -eq 0 ]; then
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_defer.log 2>&1 && \
  DV_DEFER=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_nodefer.log 2>&1
  rc=$?
  tail -1 gpurun_out/bench_defer.log | cut -c1-200; tail -1 gpurun_out/bench_nodefer.log | cut -c1-200
fi
exit $rc
