# Data-parallel path on one GPU: 2 ranks over gloo sharing the card (RCCL needs one GPU per rank).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export DV_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29533 tools/ddp_gpu_check.py > gpurun_out/ddp_check.log 2>&1
echo "ddp_check rc=$?"; grep "rank" gpurun_out/ddp_check.log | grep losses
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29534 bench.py --gpus 2 --steps 5 --warmup 2 --batch 32 > gpurun_out/bench_dp2.log 2>&1
echo "bench dp2 rc=$?"; grep metric gpurun_out/bench_dp2.log
