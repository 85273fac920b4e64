# PMC counters of the conv kernels on selected ResNet-50 layers (one pass per counter group)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/pmc
L=s2_1x1_128_512,s4_3x3_512,s1_1x1_64_256,s2_3x3_128
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pmc/t -o run --output-format csv -- python3 $R/tools/bench_conv.py --layers $L --variants 0 --iters 3 > $R/gpurun_out/pmc/t.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc/p1 -o run --output-format csv -- python3 $R/tools/bench_conv.py --layers $L --variants 0 --iters 3 > $R/gpurun_out/pmc/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES SQ_INSTS_VMEM TCC_HIT TCC_MISS -d $R/gpurun_out/pmc/p2 -o run --output-format csv -- python3 $R/tools/bench_conv.py --layers $L --variants 0 --iters 3 > $R/gpurun_out/pmc/p2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum -d $R/gpurun_out/pmc/p3 -o run --output-format csv -- python3 $R/tools/bench_conv.py --layers $L --variants 0 --iters 3 > $R/gpurun_out/pmc/p3.log 2>&1
rc=$?
echo rc=$rc
ls -R $R/gpurun_out/pmc | head -30
exit $rc
