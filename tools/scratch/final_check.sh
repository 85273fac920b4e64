#!/bin/bash
mkdir -p gpurun_out/fc
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "graph or branch or ddp or bench or determin or conv" > gpurun_out/fc/tests.log 2>&1 && \
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/fc/resnet.log 2>&1 && \
timeout -k 10 240 python bench.py --graph --steps 20 --warmup 5 > gpurun_out/fc/resnet_graph.log 2>&1 && \
timeout -k 10 240 python bench.py --model hourglass --graph --steps 20 --warmup 5 > gpurun_out/fc/hg_graph.log 2>&1 && \
timeout -k 10 240 python bench.py --model yolov3 --steps 20 --warmup 5 > gpurun_out/fc/yolo.log 2>&1 && \
timeout -k 10 240 python bench.py --model yolov3 --graph --steps 20 --warmup 5 > gpurun_out/fc/yolo_graph.log 2>&1
rc=$?
tail -2 gpurun_out/fc/tests.log; grep -E "^FAILED" gpurun_out/fc/tests.log | head
for f in resnet resnet_graph hg_graph yolo yolo_graph; do echo "$f: $(grep '^{' gpurun_out/fc/$f.log | tail -1 | grep -o '"value": [0-9.]*')"; done
exit $rc
