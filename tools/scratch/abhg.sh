set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
run() { env $1 timeout -k 10 300 python bench.py --model $2 --steps 10 --warmup 3 $3 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 $2 $3', d['value'])"; }
for i in 1 2; do for v in 0 1; do run DV_WGRAD_SIDE=$v hourglass "" || exit 1; run DV_WGRAD_SIDE=$v yolov3 "" || exit 1; done; done
