# Full GPU check: gpu tests, smoke, 1-GPU bench (native + torch/MIOpen reference), loss curve.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --backend torch > gpurun_out/bench_torch.log 2>&1 && \
timeout -k 10 300 python tools/loss_curve.py resnet50 64 20 0.1 > gpurun_out/loss_curve.log 2>&1
rc=$?
echo rc=$rc
tail -3 gpurun_out/tests.log; tail -1 gpurun_out/bench.log; tail -1 gpurun_out/bench_torch.log; cat gpurun_out/loss_curve.log
exit $rc
