set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for i in 1 2; do
for v in 0 1; do
  DV_MAIN_PRIO=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/prio_$v.log 2>&1 || exit $?
  echo "prio=$v $(tail -1 gpurun_out/prio_$v.log | cut -c1-150)"
done; done
