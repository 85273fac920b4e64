set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_heads_gpu.py -q -m gpu > gpurun_out/heads.log 2>&1
r=$?
echo "heads exit $r"
if [ $r -ne 0 ] && [ $r -ne 1 ]; then exit $r; fi
timeout -k 10 400 python -m pytest tests/test_ops_gpu.py -q -m gpu -x > gpurun_out/ops.log 2>&1
echo "ops exit $?"
tail -3 gpurun_out/heads.log gpurun_out/ops.log
