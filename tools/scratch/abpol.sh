set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
run() { env DV_WGRAD_SIDE=$1 timeout -k 10 300 python bench.py --model $2 $3 --steps 10 --warmup 3 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2 $3 side=$1', d['value'])"; }
for i in 1 2; do for v in 0 1 all; do run $v resnet50 "" || exit 1; done; done
for i in 1 2; do for v in 0 1; do run $v mobilenet1 --graph || exit 1; run $v hourglass --graph || exit 1; run $v yolov3 --graph || exit 1; done; done
