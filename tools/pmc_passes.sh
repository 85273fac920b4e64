#!/bin/bash
# PMC counter passes (one rocprofv3 run per counter group, each under its own time limit) over one
# python command line; summary via tools/pmc_summary.py.
#   bash tools/pmc_passes.sh OUTDIR PATTERN -- python3 tools/bench_conv.py ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$1; pat=$2; shift 2; [ "$1" = "--" ] && shift
mkdir -p "$R/$out"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
P2="SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU TCC_HIT TCC_MISS"
P3="FETCH_SIZE TA_BUSY_avr"
P4="WRITE_SIZE"
i=0
for pc in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pc -d "$R/$out/p$i" -o run --output-format csv -- "$@" > "$R/$out/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
cd "$R"
python tools/pmc_summary.py "$pat" $(find "$out" -name '*counter_collection.csv' | sort) > "$out/summary.txt" 2>&1
cat "$out/summary.txt" | grep -v "^ *SQ_\|^ *GRBM\|^ *TCC\|^ *FETCH" | head -60
