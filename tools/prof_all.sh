#!/bin/bash
# kernel tables of the BASELINE models in their default modes (tools/gpu.sh prof)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/tables
bash tools/gpu.sh prof resnet50 > /dev/null 2>&1 && cp gpurun_out/step_resnet50.txt gpurun_out/tables/ && \
GRAPH=1 bash tools/gpu.sh prof yolov3 > /dev/null 2>&1 && cp gpurun_out/step_yolov3_graph.txt gpurun_out/tables/ && \
GRAPH=1 bash tools/gpu.sh prof hourglass > /dev/null 2>&1 && cp gpurun_out/step_hourglass_graph.txt gpurun_out/tables/ && \
GRAPH=1 bash tools/gpu.sh prof mobilenet1 > /dev/null 2>&1 && cp gpurun_out/step_mobilenet1_graph.txt gpurun_out/tables/
rc=$?
for f in gpurun_out/tables/*.txt; do head -4 $f; done
exit $rc
