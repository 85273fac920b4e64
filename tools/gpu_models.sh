# BASELINE.json model configs on one GPU (native vs torch/MIOpen) + ResNet-50 kernel profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for m in mobilenet1 yolov3 hourglass; do
  timeout -k 10 300 python bench.py --model $m --steps 10 --warmup 3 > gpurun_out/bench_$m.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --model $m --steps 10 --warmup 3 --backend torch > gpurun_out/bench_${m}_torch.log 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r50 -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/prof_r50.log 2>&1
rc=$?
cd $R
for f in gpurun_out/bench_*.log; do echo "$f: $(tail -1 $f | cut -c1-200)"; done
echo rc=$rc
exit $rc
