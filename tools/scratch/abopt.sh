#!/bin/bash
# same-box A/B: models' weight-gradient side-stream opt-out honoured (1) vs ignored (0), 8 HW queues
mkdir -p gpurun_out/abopt; rc=0
for spec in "mobilenet1 --graph" "hourglass --graph" "mobilenet1" ; do
  set -- $spec; m=$1; shift; a="$*"
  for i in 1 2; do for s in 1 0; do
    [ $rc -eq 0 ] || break
    DV_WGRAD_SIDE_OPTOUT=$s timeout -k 10 240 python bench.py --model $m $a --steps 20 --warmup 5 > gpurun_out/abopt/${m}${a// /}_${s}_$i.log 2>&1 || rc=$?
    echo "$m $a OPTOUT=$s run $i: $(grep '^{' gpurun_out/abopt/${m}${a// /}_${s}_$i.log | tail -1 | cut -c1-120)"
  done; done
done
exit $rc
