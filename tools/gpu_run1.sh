set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -c "import torch;print(torch.cuda.get_device_name(0), torch.version.hip)" > gpurun_out/dev.log 2>&1
timeout -k 10 400 python -m pytest tests/test_ops_gpu.py -q -m gpu > gpurun_out/t1.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench1.log 2>&1
