set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
run() { env $1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 $2 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 $2', d['value'])"; }
for i in 1 2; do
  run "DV_WGRAD_SIDE_DP=0" --force-dp || exit 1
  run "DV_WGRAD_SIDE_DP=1 GPU_MAX_HW_QUEUES=8" --force-dp || exit 1
  run "DV_WGRAD_SIDE_DP=1 GPU_MAX_HW_QUEUES=16" --force-dp || exit 1
  run "GPU_MAX_HW_QUEUES=8" "" || exit 1
done
