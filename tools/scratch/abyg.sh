#!/bin/bash
mkdir -p gpurun_out/abyg; rc=0
for m in yolov3 resnet50; do for i in 1 2; do for s in 0 1; do
  [ $rc -eq 0 ] && { DV_WGRAD_SIDE_GRAPH=$s timeout -k 10 240 python bench.py --model $m --graph --steps 30 --warmup 5 > gpurun_out/abyg/${m}_${s}_$i.log 2>&1 || rc=$?; }
done; done; done
[ $rc -eq 0 ] && { timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_graph_gpu.py tests/test_branch_streams_gpu.py > gpurun_out/abyg/tests.log 2>&1 || rc=$?; }
for f in gpurun_out/abyg/*_*.log; do echo "$(basename $f .log): $(grep '^{' $f | tail -1 | grep -o '"value": [0-9.]*')"; done
tail -1 gpurun_out/abyg/tests.log
exit $rc
