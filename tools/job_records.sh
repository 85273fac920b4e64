#!/bin/bash
# refresh the native bench records (eager + graph) of the BASELINE GPU configs
mkdir -p gpurun_out/rec
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/rec/resnet50_eager.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph > gpurun_out/rec/resnet50_graph.log 2>&1 || exit $?
for m in mobilenet1 hourglass yolov3; do
  s=20; [ $m != mobilenet1 ] && s=10
  timeout -k 10 300 python bench.py --model $m --steps $s --warmup 3 > gpurun_out/rec/${m}_eager.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --model $m --steps $s --warmup 3 --graph > gpurun_out/rec/${m}_graph.log 2>&1 || exit $?
done
for f in gpurun_out/rec/*.log; do echo "$f $(grep '^{' $f | tail -1 | cut -c1-150)"; done
