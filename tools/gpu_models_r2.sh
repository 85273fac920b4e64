#!/bin/bash
# Bench every BASELINE model config (native and torch/MIOpen) + kernel profiles of vgg16 / mobilenet1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
rc=0
for m in ${MODELS:-mobilenet1 yolov3 hourglass vgg16 inception1}; do
  timeout -k 10 300 python bench.py --model $m --steps 10 --warmup 3 > gpurun_out/bench_$m.log 2>&1 || { rc=$?; break; }
  timeout -k 10 300 python bench.py --model $m --steps 10 --warmup 3 --backend torch > gpurun_out/bench_${m}_torch.log 2>&1 || { rc=$?; break; }
done
for f in gpurun_out/bench_*.log; do echo "$f: $(tail -1 $f | cut -c1-180)"; done
[ $rc -ne 0 ] && exit $rc
for m in ${PROF:-vgg16 mobilenet1}; do
  bash tools/gpu.sh prof $m > /dev/null 2>&1 || exit $?
  head -14 gpurun_out/prof_$m.txt
done
