#!/bin/bash
# Same-box bench A/B of one env switch: AB=VAR VALS="a b" MODEL=m ARGS="..." REPS=2 tools/ab_env.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
for r in $(seq ${REPS:-2}); do
  for v in $VALS; do
    env $AB=$v timeout -k 10 300 python bench.py --model ${MODEL:-resnet50} $ARGS > gpurun_out/ab_${v}.log 2>&1 || exit $?
    echo "$AB=$v $(tail -1 gpurun_out/ab_${v}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
