#!/bin/bash
# Round-4 evidence: steady-state kernel tables (ResNet-50 eager, MobileNet / Hourglass / YOLOv3 graph),
# conv-vs-MIOpen per-layer table; stops at the first crash / timeout
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
bash tools/gpu.sh prof resnet50 > gpurun_out/j_prof_rn.log 2>&1 || exit $?
tail -45 gpurun_out/step_resnet50.txt | head -14
for m in mobilenet1 hourglass yolov3; do
  GRAPH=1 bash tools/gpu.sh prof $m > gpurun_out/j_prof_$m.log 2>&1 || exit $?
  head -14 gpurun_out/step_${m}_graph.txt
done
timeout -k 10 600 python -u tools/conv_vs_miopen.py --iters 10 --out gpurun_out/conv_vs_miopen.txt > gpurun_out/conv_vs_miopen.log 2>&1 || exit $?
cat gpurun_out/conv_vs_miopen.txt
cd /tmp && timeout 200 hipcc --offload-arch=gfx950 -O3 "$R/tools/mfma_shape_bench.hip" -o /tmp/mfma_shape_bench && cd "$R" && \
  timeout -k 5 60 /tmp/mfma_shape_bench > gpurun_out/mfma_shape.txt 2>&1 || exit $?
cat gpurun_out/mfma_shape.txt
PMC_ARGS=--wgrad bash tools/gpu.sh pmc s1_3x3_64,s2_3x3_128,s3_3x3_256,s4_3x3_512 conv_wgrad > gpurun_out/j_pmc_wg.log 2>&1 || exit $?
cp -r gpurun_out/pmc/summary.txt gpurun_out/pmc_wgrad_r4.txt
bash tools/gpu.sh pmc s1_3x3_64,s2_3x3_128,s3_3x3_256,s4_3x3_512,s2_1x1_128_512 conv_fwd > gpurun_out/j_pmc_fw.log 2>&1 || exit $?
cp -r gpurun_out/pmc/summary.txt gpurun_out/pmc_fwd_r4.txt
head -40 gpurun_out/pmc_wgrad_r4.txt
