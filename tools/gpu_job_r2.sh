set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread ${TESTS:-tests} -m gpu > gpurun_out/tests.log 2>&1
rc=$?; tail -3 gpurun_out/tests.log; grep -E "FAILED|Error" gpurun_out/tests.log | head -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log | cut -c1-250 && \
timeout -k 10 300 python tools/loss_curve.py resnet50 128 100 0.01 learnable gpurun_out/loss_curve_resnet50.json > gpurun_out/lc_r50.log 2>&1 && \
timeout -k 10 300 python tools/loss_curve.py mobilenet1 128 100 0.02 learnable gpurun_out/loss_curve_mobilenet1.json > gpurun_out/lc_mb.log 2>&1
rc=$?; cat gpurun_out/lc_r50.log gpurun_out/lc_mb.log | grep -v amdgpu.ids | cut -c1-200; exit $rc
