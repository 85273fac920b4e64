set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
run() { env $1 timeout -k 10 300 python bench.py --model mobilenet1 --steps 20 --warmup 5 $2 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 $2', d['value'])"; }
for i in 1 2; do for v in 0 1; do run DV_DW_WGRAD_SIDE=$v --graph || exit 1; run DV_DW_WGRAD_SIDE=$v "" || exit 1; done; done
