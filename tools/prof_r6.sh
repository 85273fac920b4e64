set -o pipefail
cd $GRAFT_REPO_ROOT
DV_WGRAD_SIDE=0 bash tools/gpu.sh prof resnet50 > /dev/null 2>&1 && mkdir -p gpurun_out/ss && cp gpurun_out/step_resnet50.txt gpurun_out/census_resnet50.txt gpurun_out/prof_resnet50.txt gpurun_out/ss/ && \
bash tools/gpu.sh prof resnet50 > /dev/null 2>&1 && \
bash tools/gpu.sh pmc s1_3x3_64,s2_3x3_128,s3_3x3_256,s4_3x3_512,s1_1x1_64_256 > /dev/null 2>&1 && cp gpurun_out/pmc/summary.txt gpurun_out/pmc_fwd_summary.txt && rm -rf gpurun_out/pmc && \
PMC_ARGS=--wgrad bash tools/gpu.sh pmc s1_3x3_64,s2_3x3_128,s3_3x3_256,s4_3x3_512,s1_1x1_64_256 conv_wgrad > /dev/null 2>&1 && cp gpurun_out/pmc/summary.txt gpurun_out/pmc_wgrad_summary.txt
rc=$?
head -30 gpurun_out/ss/step_resnet50.txt; head -30 gpurun_out/step_resnet50.txt
exit $rc
