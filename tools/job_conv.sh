#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 1100 python -u tools/convergence.py --steps 1000 --seeds 0 1 --every 100 --out gpurun_out/convergence_resnet50.json > gpurun_out/convergence.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/convergence.log | tail -50; exit $rc
