#!/bin/bash
# fused BN finalize A/B: benches (off / atomic-exchange fold / atomic-load fold) + kernel traces
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
DV_FIN_LOADS=1 timeout -k 10 300 $PYT tests/test_bn_finalize_fused_gpu.py > gpurun_out/fin2_tests.log 2>&1 && \
DV_FUSE_FINALIZE=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/fin2_off.log 2>&1 && \
DV_FUSE_FINALIZE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/fin2_exch.log 2>&1 && \
DV_FUSE_FINALIZE=1 DV_FIN_LOADS=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/fin2_loads.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
for v in off exch loads; do
  e="DV_FUSE_FINALIZE=1"; [ $v = off ] && e="DV_FUSE_FINALIZE=0"; [ $v = loads ] && e="DV_FUSE_FINALIZE=1 DV_FIN_LOADS=1"
  env $e timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/fin2_prof_$v" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps 6 --warmup 2 > "$R/gpurun_out/fin2_prof_$v.log" 2>&1 || exit $?
  t=$(find "$R/gpurun_out/fin2_prof_$v" -name '*kernel_trace.csv' -print -quit)
  python "$R/tools/step_table.py" "$t" --steps 4 --title "resnet50 fin=$v" > "$R/gpurun_out/fin2_step_$v.txt" 2>&1
  rm -f "$t"
done
rc=$?
cd "$R"
tail -2 gpurun_out/fin2_tests.log
for f in gpurun_out/fin2_*.log; do echo "$f: $(grep '^{' $f | tail -1 | cut -c1-110)"; done
for v in off exch loads; do sed -n 3,12p gpurun_out/fin2_step_$v.txt; done
exit $rc
