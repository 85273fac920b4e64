#!/bin/bash
# Same-box A/B of ./ab_old (tools/ab_tree.sh <commit>) against the working tree over several
# models: MODELS="resnet50 yolov3" REPS=2 tools/ab_models.sh   (bench.py defaults per model)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/abm
[ -d ab_old ] || { echo "no ab_old/ (run tools/ab_tree.sh <commit> first)"; exit 2; }
val() { grep '^{' "$1" | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for m in ${MODELS:-resnet50}; do
  for i in $(seq ${REPS:-1}); do
    (cd ab_old && timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5) > gpurun_out/abm/old_${m}_$i.log 2>&1 || exit $?
    timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/abm/new_${m}_$i.log 2>&1 || exit $?
    echo "$m old $(val gpurun_out/abm/old_${m}_$i.log)   new $(val gpurun_out/abm/new_${m}_$i.log)"
  done
done
