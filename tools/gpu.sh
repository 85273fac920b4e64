#!/bin/bash
# One entry point for every GPU-box job (run through gpurun from the repo root):
#   tools/gpu.sh check           GPU tests, smoke, 1-GPU ResNet-50 bench
#   tools/gpu.sh bench [args]    bench.py with the given args (default ResNet-50, 1 GPU)
#   tools/gpu.sh prof MODEL      rocprofv3 kernel trace + stats of bench.py --model MODEL
#   tools/gpu.sh pmc  LAYERS [PAT] PMC counter passes (one run per counter group) over tools/bench_conv.py layers
#                                (PMC_ARGS=--wgrad for the weight-gradient kernels; PAT filters kernel names)
#   tools/gpu.sh models          bench every BASELINE.json GPU config (native and torch/MIOpen reference)
#   tools/gpu.sh tests [-k EXPR] GPU tests only
#   tools/gpu.sh records         eager + graph bench records of the BASELINE GPU configs
#   tools/gpu.sh evidence        kernel tables of the four BASELINE models + conv-vs-MIOpen table
#   tools/gpu.sh host            Python host profiles of the eager launch-bound models
#   tools/gpu.sh convergence     ResNet-50 1,000-step native vs torch-bf16 curves, 2 seeds
#   tools/gpu.sh overlap         DP bucket overlap test + force-DP kernel timeline
#   AB=VAR [MODEL=m ARGS=..] tools/gpu.sh ab   same-box bench + kernel-trace A/B of an env toggle
#   tools/gpu.sh abtree          same-box bench A/B of ./ab_old (tools/ab_tree.sh <commit>) vs the tree
# Every GPU step has its own time limit and the steps are chained with &&: after a fault,
# abort or timeout nothing else runs on the GPU in that call.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
mode=${1:-check}; shift || true
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
case "$mode" in
  check)
    timeout -k 10 900 $PYT tests -m gpu > gpurun_out/tests.log 2>&1 && \
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 && \
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --force-dp > gpurun_out/bench_dp1.log 2>&1
    rc=$?; tail -3 gpurun_out/tests.log; grep -E "^FAILED" gpurun_out/tests.log | head
    tail -1 gpurun_out/bench.log | cut -c1-300; tail -1 gpurun_out/bench_dp1.log | cut -c1-300 ;;
  tests)
    timeout -k 10 900 $PYT tests -m gpu "$@" > gpurun_out/tests.log 2>&1
    rc=$?; grep -E "PASSED|FAILED|ERROR" gpurun_out/tests.log | tail -40; tail -3 gpurun_out/tests.log ;;
  bench)
    timeout -k 10 400 python bench.py "$@" > gpurun_out/bench.log 2>&1
    rc=$?; tail -1 gpurun_out/bench.log | cut -c1-400 ;;
  prof)
    # GRAPH=1: profile the HIP-graph replay step (bench.py --graph); BATCH=n overrides the batch
    m=${1:-resnet50}
    extra=""; [ -n "$GRAPH" ] && extra="--graph"; [ -n "$BATCH" ] && extra="$extra --batch $BATCH"
    tag=$m${GRAPH:+_graph}
    cd /tmp && export TMPDIR=/tmp && \
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$tag" -o run --output-format csv -- \
      python3 "$R/bench.py" --model "$m" --steps 6 --warmup 2 $extra > "$R/gpurun_out/prof_$tag.log" 2>&1
    rc=$?; cd "$R"
    f=$(find gpurun_out/prof_$tag -name '*kernel_stats.csv' -print -quit)
    [ -n "$f" ] && python tools/prof_summary.py "$f" 8 "$m bench.py --steps 6 --warmup 2 $extra" > gpurun_out/prof_$tag.txt 2>&1
    t=$(find gpurun_out/prof_$tag -name '*kernel_trace.csv' -print -quit)
    [ -n "$t" ] && python tools/step_table.py "$t" --steps 4 --title "$m bench.py $extra (rocprofv3 --kernel-trace)" > gpurun_out/step_$tag.txt 2>&1
    [ -n "$t" ] && python tools/trace_step.py "$t" > gpurun_out/trace_$tag.txt 2>&1
    [ -n "$t" ] && python tools/kernel_census.py "$t" > gpurun_out/census_$tag.txt 2>&1
    rm -f "$t"
    cat gpurun_out/step_$tag.txt | cut -c1-160 | sed -n '1,45p' ;;
  pmc)
    L=${1:-s2_1x1_128_512,s4_3x3_512,s1_1x1_64_256,s2_3x3_128}
    mkdir -p gpurun_out/pmc && cd /tmp && export TMPDIR=/tmp && \
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d "$R/gpurun_out/pmc/p1" -o run --output-format csv -- python3 "$R/tools/bench_conv.py" --layers "$L" --variants 0 --iters 3 $PMC_ARGS > "$R/gpurun_out/pmc/p1.log" 2>&1 && \
    timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM TCC_HIT TCC_MISS -d "$R/gpurun_out/pmc/p2" -o run --output-format csv -- python3 "$R/tools/bench_conv.py" --layers "$L" --variants 0 --iters 3 $PMC_ARGS > "$R/gpurun_out/pmc/p2.log" 2>&1 && \
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TA_BUSY_avr -d "$R/gpurun_out/pmc/p3" -o run --output-format csv -- python3 "$R/tools/bench_conv.py" --layers "$L" --variants 0 --iters 3 $PMC_ARGS > "$R/gpurun_out/pmc/p3.log" 2>&1
    rc=$?; cd "$R"
    python tools/pmc_summary.py "${2:-conv_}" $(find gpurun_out/pmc -name '*counter_collection.csv') > gpurun_out/pmc/summary.txt 2>&1
    sed -n '1,80p' gpurun_out/pmc/summary.txt ;;
  models)
    rc=0
    for m in mobilenet1 yolov3 hourglass; do
      timeout -k 10 300 python bench.py --model $m --steps 10 --warmup 3 > gpurun_out/bench_$m.log 2>&1 || { rc=$?; break; }
      timeout -k 10 300 python bench.py --model $m --steps 10 --warmup 3 --backend torch > gpurun_out/bench_${m}_torch.log 2>&1 || { rc=$?; break; }
    done
    for f in gpurun_out/bench_*.log; do echo "$f: $(tail -1 $f | cut -c1-200)"; done ;;
  pmcdw)
    # PMC passes over the depthwise kernels (tools/dw_bench.py, variant 0)
    mkdir -p gpurun_out/pmcdw && cd /tmp && export TMPDIR=/tmp && \
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d "$R/gpurun_out/pmcdw/p1" -o run --output-format csv -- python3 "$R/tools/dw_bench.py" --variants 0 --iters 3 > "$R/gpurun_out/pmcdw/p1.log" 2>&1 && \
    timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU TCC_HIT TCC_MISS GRBM_GUI_ACTIVE -d "$R/gpurun_out/pmcdw/p2" -o run --output-format csv -- python3 "$R/tools/dw_bench.py" --variants 0 --iters 3 > "$R/gpurun_out/pmcdw/p2.log" 2>&1 && \
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TA_BUSY_avr -d "$R/gpurun_out/pmcdw/p3" -o run --output-format csv -- python3 "$R/tools/dw_bench.py" --variants 0 --iters 3 > "$R/gpurun_out/pmcdw/p3.log" 2>&1
    rc=$?; cd "$R"
    python tools/pmc_summary.py "dw_" $(find gpurun_out/pmcdw -name '*counter_collection.csv') > gpurun_out/pmcdw/summary.txt 2>&1
    sed -n '1,60p' gpurun_out/pmcdw/summary.txt ;;
  zoo)
    # per-model bench, native and PyTorch/MIOpen arms (MODELS overrides the list)
    rc=0
    for m in ${MODELS:-resnet50 inception1 alexnet2 vgg16 shufflenet1}; do
      timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/bench_$m.log 2>&1 || { rc=$?; break; }
      timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 --backend torch > gpurun_out/bench_${m}_torch.log 2>&1 || { rc=$?; break; }
    done
    for f in gpurun_out/bench_*.log; do echo "$f: $(grep '^{' $f | tail -1 | cut -c1-160)"; done ;;
  lc)
    timeout -k 10 600 python tools/lc_sweep.py --models ${MODELS:-resnet50} --grid ${GRID:-0.05:1.0,0.02:1.0} \
      --out gpurun_out/lc_sweep.txt > gpurun_out/lc_sweep.log 2>&1
    rc=$?; cat gpurun_out/lc_sweep.log | cut -c1-200 ;;
  records)
    # native bench records (eager + graph) of the BASELINE GPU configs -> gpurun_out/rec/*.log
    mkdir -p gpurun_out/rec; rc=0
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/rec/resnet50_eager.log 2>&1 && \
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph > gpurun_out/rec/resnet50_graph.log 2>&1 || rc=$?
    for m in mobilenet1 hourglass yolov3; do
      [ $rc -ne 0 ] && break
      s=20; [ $m != mobilenet1 ] && s=10
      timeout -k 10 300 python bench.py --model $m --steps $s --warmup 3 > gpurun_out/rec/${m}_eager.log 2>&1 && \
      timeout -k 10 300 python bench.py --model $m --steps $s --warmup 3 --graph > gpurun_out/rec/${m}_graph.log 2>&1 || rc=$?
    done
    for f in gpurun_out/rec/*.log; do echo "$f $(grep '^{' $f | tail -1 | cut -c1-150)"; done ;;
  evidence)
    # steady-state kernel tables (ResNet-50 eager, MobileNet / Hourglass / YOLOv3 graph) and the
    # per-layer conv-vs-MIOpen table
    bash tools/gpu.sh prof resnet50 > gpurun_out/j_prof_rn.log 2>&1 && \
    GRAPH=1 bash tools/gpu.sh prof mobilenet1 > gpurun_out/j_prof_mb.log 2>&1 && \
    GRAPH=1 bash tools/gpu.sh prof hourglass > gpurun_out/j_prof_hg.log 2>&1 && \
    GRAPH=1 bash tools/gpu.sh prof yolov3 > gpurun_out/j_prof_yl.log 2>&1 && \
    timeout -k 10 600 python -u tools/conv_vs_miopen.py --iters 10 --out gpurun_out/conv_vs_miopen.txt > gpurun_out/conv_vs_miopen.log 2>&1
    rc=$?; for f in gpurun_out/step_*.txt; do head -3 $f; done ;;
  host)
    # host-side (Python) profiles of the eager launch-bound models
    timeout -k 10 300 python tools/host_profile.py --model hourglass --steps 5 --top 45 > gpurun_out/host_hourglass.txt 2>&1 && \
    timeout -k 10 300 python tools/host_profile.py --model yolov3 --steps 5 --top 45 > gpurun_out/host_yolov3.txt 2>&1
    rc=$?; head -14 gpurun_out/host_hourglass.txt | cut -c1-150 ;;
  convergence)
    # ResNet-50 1,000 steps x 2 seeds, native vs torch autocast-bf16 (tools/convergence.py)
    timeout -k 10 1100 python -u tools/convergence.py --steps 1000 --seeds 0 1 --every 100 \
      --out gpurun_out/convergence_resnet50.json > gpurun_out/convergence.log 2>&1
    rc=$?; grep -v amdgpu.ids gpurun_out/convergence.log | tail -50 ;;
  overlap)
    # bucket all-reduce overlap evidence (world-1 RCCL, DataParallel forced on): the issue-order GPU
    # test, then a kernel trace of the force-DP ResNet-50 step summarised by tools/comm_timeline.py
    timeout -k 10 400 $PYT -s tests/test_ddp_gpu.py -k overlap > gpurun_out/overlap_test.log 2>&1 && \
    cd /tmp && export TMPDIR=/tmp && \
    timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/gpurun_out/prof_dp" -o run --output-format csv -- \
      python3 "$R/bench.py" --force-dp --bucket-mb 8 --steps 3 --warmup 2 > "$R/gpurun_out/prof_dp.log" 2>&1
    rc=$?; cd "$R"
    t=$(find gpurun_out/prof_dp -name '*kernel_trace.csv' -print -quit 2>/dev/null)
    [ -n "$t" ] && python tools/comm_timeline.py "$t" > gpurun_out/comm_timeline.txt 2>&1; rm -f "$t"
    grep -E "PASS|FAIL|backward .* ms" gpurun_out/overlap_test.log | head; head -40 gpurun_out/comm_timeline.txt 2>/dev/null ;;
  ab)
    # same-box A/B of an environment toggle: bench.py alternating off / on twice, then a kernel
    # trace of each arm:  AB=DV_FUSE_FIN MODEL=hourglass ARGS=--graph tools/gpu.sh ab
    v=${AB:?set AB=VAR}; m=${MODEL:-resnet50}; args=${ARGS:-}
    rc=0
    for i in 1 2; do for s in 0 1; do
      [ $rc -eq 0 ] && { env $v=$s timeout -k 10 300 python bench.py --model $m $args --steps 10 --warmup 3 > gpurun_out/ab_${s}_$i.log 2>&1 || rc=$?; }
    done; done
    [ $rc -eq 0 ] && cd /tmp && export TMPDIR=/tmp && \
    env $v=0 timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/ab_prof_0" -o run --output-format csv -- \
      python3 "$R/bench.py" --model $m $args --steps 6 --warmup 2 > "$R/gpurun_out/ab_prof_0.log" 2>&1 && \
    env $v=1 timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/ab_prof_1" -o run --output-format csv -- \
      python3 "$R/bench.py" --model $m $args --steps 6 --warmup 2 > "$R/gpurun_out/ab_prof_1.log" 2>&1
    rc=$?; cd "$R"
    for s in 0 1; do
      t=$(find gpurun_out/ab_prof_$s -name '*kernel_trace.csv' -print -quit 2>/dev/null)
      [ -n "$t" ] && python tools/step_table.py "$t" --steps 4 --title "$m $args $v=$s" > gpurun_out/ab_step_$s.txt 2>&1
      rm -f "$t"
      for i in 1 2; do echo "$v=$s run $i: $(grep '^{' gpurun_out/ab_${s}_$i.log | tail -1 | cut -c1-110)"; done
      sed -n 1,14p gpurun_out/ab_step_$s.txt 2>/dev/null
    done ;;
  abtree)
    # same-box A/B of the tree in ./ab_old (tools/ab_tree.sh <commit>) against the working tree:
    # ResNet-50 eager, alternating old / new twice, then MobileNet --graph once each
    [ -d ab_old ] || { echo "no ab_old/ (run tools/ab_tree.sh <commit> first)"; exit 2; }
    mkdir -p gpurun_out/abx; rc=0
    for i in 1 2; do
      (cd ab_old && timeout -k 10 300 python bench.py --steps 20 --warmup 5) > gpurun_out/abx/old_$i.log 2>&1 && \
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/abx/new_$i.log 2>&1 || { rc=$?; break; }
    done
    [ $rc -eq 0 ] && { (cd ab_old && timeout -k 10 300 python bench.py --model mobilenet1 --graph --steps 20 --warmup 3) \
      > gpurun_out/abx/old_mb.log 2>&1 && timeout -k 10 300 python bench.py --model mobilenet1 --graph --steps 20 \
      --warmup 3 > gpurun_out/abx/new_mb.log 2>&1 || rc=$?; }
    for f in gpurun_out/abx/*.log; do echo "$f $(grep '^{' $f | tail -1 | cut -c1-110)"; done ;;
  *) echo "unknown mode $mode"; exit 2 ;;
esac
echo "rc=$rc"
exit $rc
