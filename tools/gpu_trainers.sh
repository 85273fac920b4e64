# Smoke-train every family on the GPU (synthetic data) + the full GPU test suite.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/tr && cd gpurun_out/tr
R=$GRAFT_REPO_ROOT
run() { local name=$1; shift; echo "== $name"; timeout -k 10 300 "$@" > $name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -4 $name.log; return $rc; }
run resnet50 python $R/ResNet/pytorch/train.py -m resnet50 --synthetic --synthetic-size 1280 --epochs 1 --max-steps 20 --val-steps 2 --batch-size 64 --workers 2 --profile --checkpoint-dir /tmp/dvck/ &&
run mobilenet python $R/MobileNet/pytorch/train.py -m mobilenet1 --synthetic --synthetic-size 640 --epochs 1 --max-steps 10 --val-steps 2 --batch-size 64 --workers 2 --checkpoint-dir /tmp/dvck/ &&
run inception python $R/Inception/pytorch/train.py -m inception1 --synthetic --synthetic-size 640 --epochs 1 --max-steps 10 --val-steps 2 --batch-size 64 --workers 2 --checkpoint-dir /tmp/dvck/ &&
run yolov3 python $R/YOLO/tensorflow/train.py --synthetic --synthetic-size 32 --epochs 1 --max-steps 4 --val-steps 2 --batch-size 8 --log-every 2 --profile --checkpoint-dir /tmp/dvck/ &&
run hourglass python $R/Hourglass/tensorflow/train.py --synthetic --synthetic-size 32 --epochs 1 --max-steps 4 --val-steps 2 --batch-size 8 --log-every 2 --checkpoint-dir /tmp/dvck/ &&
run centernet python $R/ObjectsAsPoints/tensorflow/train.py --synthetic --synthetic-size 16 --epochs 1 --max-steps 4 --val-steps 2 --batch-size 4 --log-every 2 --checkpoint-dir /tmp/dvck/ &&
run dcgan python $R/DCGAN/tensorflow/main.py --synthetic --epochs 2 --max-steps 5 --checkpoint-dir /tmp/dvck/dc &&
run cyclegan python $R/CycleGAN/tensorflow/train.py --dataset toy --synthetic --epochs 2 --max-steps 2 --batch_size 1 --checkpoint-dir /tmp/dvck/cg &&
cd $R && echo "== pytest gpu" && timeout -k 10 600 python -m pytest tests -q -m gpu > gpurun_out/tests.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/tests.log
