#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
bash tools/gpu.sh prof resnet50 > gpurun_out/j_prof_rn.log 2>&1 || exit $?
head -14 gpurun_out/step_resnet50.txt
for m in hourglass mobilenet1 yolov3; do
  GRAPH=1 bash tools/gpu.sh prof $m > gpurun_out/j_prof_$m.log 2>&1 || exit $?
  head -14 gpurun_out/step_${m}_graph.txt
done
