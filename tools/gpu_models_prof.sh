# full GPU tests + kernel profiles of the YOLOv3 and Hourglass training steps
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_yolo -o run --output-format csv -- python3 $R/bench.py --model yolov3 --steps 5 --warmup 2 > $R/gpurun_out/prof_yolo.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_hg -o run --output-format csv -- python3 $R/bench.py --model hourglass --steps 5 --warmup 2 > $R/gpurun_out/prof_hg.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_mb -o run --output-format csv -- python3 $R/bench.py --model mobilenet1 --steps 5 --warmup 2 > $R/gpurun_out/prof_mb.log 2>&1
rc=$?
cd $R
tail -2 gpurun_out/tests.log
echo rc=$rc
exit $rc
