#!/usr/bin/env python3
"""Training-throughput benchmark (images/sec, whole job) for the BASELINE.json configs.

Default / flagship: ResNet-50 V1 bf16 224x224, synthetic ImageNet-shaped data, random-init
weights, SGD(lr .1, momentum .9, wd 1e-4) as R/ResNet/pytorch/train.py:166-184, per-GPU batch
256 (weak scaling), data parallel over RCCL with one process per GPU.

Other BASELINE.json configs (``--model``):
  mobilenet1  MobileNet V1 1.0, depthwise HIP path, RMSprop(.045, .9, eps 1) per-GPU batch 128
              (R/ResNet/pytorch/train.py:185-214)
  yolov3      YOLOv3-80 416x416, synthetic COCO-shaped boxes -> 3-scale labels, YoloLoss,
              Adam(.01), 16 images per replica (R/YOLO/tensorflow/train.py:13-19,46-68)
  hourglass   Stacked Hourglass-104 (4 stacks, 16 heatmaps) 256x256, synthetic MPII-shaped
              heatmaps, weighted MSE, Adam(1e-3), 32 per replica (R/Hourglass/tensorflow/main.py:22-33)
  lenet5      LeNet-5 1x32x32 on the CPU (plumbing config), Adam(1e-3), batch 64

Every timed step is a full training step: forward, loss, backward, bucketed gradient
all-reduce (N > 1), fused optimizer update, gradient zeroing. Inputs/labels are generated once
on the device (synthetic, no host pipeline in the timed region).

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--model resnet50]
  N > 1: either launched by the driver as ``torch.distributed.run --nproc-per-node N bench.py
  --gpus N`` (one rank per GPU, RCCL), or run directly: ``bench.py --gpus N`` then spawns the N
  ranks itself (deep_vision_amd.launch, a child ``torch.distributed.run`` on 127.0.0.1) BEFORE
  touching the GPU and exits with the children's status -- it never measures 1 GPU while
  claiming N.

Reported besides the contract fields: ``per_gpu`` images/s, ``comm_exposed_ms`` (compute-stream
time blocked on the gradient all-reduces per step, HIP events around DataParallel.finish) and
``vs_same_box_miopen`` (ratio to the PyTorch/MIOpen eager run on the same MI355X, read from the
record ``bench.py --backend torch --write-comparator`` measured, bench/comparators/bench_<model>_1gpu_torch_miopen.json
-- outside the gpurun-ignored profiles/, so it travels to the GPU box -- scaled by N; the file is
named in ``vs_same_box_miopen_src``). ``vs_baseline`` divides by the
BASELINE.md proxy (~376 img/s per 8-GPU node, fp32 K80-era); it is NOT a like-for-like ratio.
"""
from __future__ import annotations

import argparse
import json
import sys
import time

# The process's step mode and hardware-queue count (deep_vision_amd/policy.py: eager steps get 8
# queues, captured steps HIP's default 4; the mode defaults to the model's measured-faster one),
# decided before torch / HIP initialise -- in this process and in every rank torchrun starts.
def _pre_args(argv):
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--graph", action=argparse.BooleanOptionalAction, default=None)
    return ap.parse_known_args(argv)[0]


_PRE = _pre_args(sys.argv[1:])
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
from deep_vision_amd import policy as _policy  # noqa: E402  (imports no torch)

GRAPH = _policy.configure(_PRE.model, _PRE.graph)

# Reference-derived comparators, images/sec per node:
#   ResNet-50-equivalent proxy ~376 (8 GPUs), YOLOv3 ~179 (8x V100), LeNet-5 PT ~906.
BASELINES = {"resnet50": 376.0, "yolov3": 179.0, "lenet5": 906.0}
ROOT = __import__("os").path.dirname(__import__("os").path.abspath(__file__))
PROFILES = __import__("os").path.join(ROOT, "profiles")
COMPARATORS = __import__("os").path.join(ROOT, "bench", "comparators")


def comparator_path(model):
    """The same-box PyTorch-ROCm eager (MIOpen) record of ``model`` on one GPU: written by
    ``bench.py --backend torch --model M`` (the measured run, not a constant), read by the native
    arm for ``vs_same_box_miopen``."""
    import os

    return os.path.join(COMPARATORS, f"bench_{model}_1gpu_torch_miopen.json")


def same_box_miopen(model):
    """(per-GPU images/s, source file) of the measured MIOpen arm, or (None, None)."""
    import os

    path = comparator_path(model)
    if not os.path.exists(path):
        return None, None
    try:
        with open(path) as f:
            rec = json.loads(f.read().strip().splitlines()[-1])
        if rec.get("config", {}).get("backend") != "torch" or not rec.get("per_gpu"):
            return None, None
        return float(rec["per_gpu"]), os.path.relpath(path, ROOT)
    except (OSError, ValueError, KeyError, IndexError):
        return None, None

RESNET_METRIC = "images/sec (whole node), ResNet-50 224x224 bf16 at 1/2/4/8 MI355X"

# model -> (per-GPU batch, image size, optimizer name, optimizer kwargs, family)
SPECS = {
    "resnet50": (256, 224, "SGD", {"lr": 0.1, "momentum": 0.9, "weight_decay": 1e-4}, "cls"),
    "resnet152": (256, 224, "SGD", {"lr": 0.1, "momentum": 0.9, "weight_decay": 1e-4}, "cls"),
    "resnet34": (256, 224, "SGD", {"lr": 0.1, "momentum": 0.9, "weight_decay": 1e-4}, "cls"),
    "mobilenet1": (128, 224, "RMSprop", {"lr": 0.045, "alpha": 0.9, "eps": 1.0}, "cls"),
    "shufflenet1": (128, 224, "RMSprop", {"lr": 0.045, "alpha": 0.9, "eps": 1.0}, "cls"),
    "vgg16": (128, 224, "SGD", {"lr": 0.01, "momentum": 0.9, "weight_decay": 5e-4}, "cls"),
    "alexnet2": (128, 224, "SGD", {"lr": 0.01, "momentum": 0.9, "weight_decay": 5e-4}, "cls"),
    "inception1": (128, 224, "SGD", {"lr": 0.01, "momentum": 0.9, "weight_decay": 2e-4}, "cls"),
    "yolov3": (16, 416, "Adam", {"lr": 0.01}, "yolo"),
    "hourglass": (32, 256, "Adam", {"lr": 1e-3}, "hourglass"),
    "lenet5": (64, 32, "Adam", {"lr": 1e-3}, "cls"),
}


def _sample_cls(i, cin, size, ncls):
    """Global sample ``i`` of the synthetic classification set (a pure function of i, so the
    global batch is the same whatever the world size: rank r holds samples [r*B, (r+1)*B))."""
    import torch

    # learnable, so the reported loss_first_last shows the step training: the label is one of
    # min(100, ncls) classes and the image that class's smooth template (an 8x8 Gaussian field,
    # upsampled) plus N(0, 0.5^2) noise -- same shapes and dtypes as random inputs
    k = min(100, ncls)
    c = i % k
    gt = torch.Generator().manual_seed(104729 * c + 3)
    t = torch.nn.functional.interpolate(torch.randn(1, cin, 8, 8, generator=gt), size=(size, size), mode="bilinear",
                                        align_corners=False)[0]
    g = torch.Generator().manual_seed(7919 * i + 17)
    return t / t.std() + 0.5 * torch.randn(cin, size, size, generator=g), c * (ncls // k)


def build_step_for_profile(model_name, batch=0):
    """(step closure, images per step) of the 1-GPU native training step of ``model_name``, as
    timed by main() (tools/host_profile.py)."""
    import torch

    from deep_vision_amd.train.optim import FusedAdam, FusedRMSprop, FusedSGD

    args = argparse.Namespace(model=model_name, batch=batch, backend="native")
    model, loss_fn, x, B, _ = build(args, torch.device("cuda"))
    _, _, opt_name, opt_kw, _ = SPECS[model_name]
    opt = {"SGD": FusedSGD, "Adam": FusedAdam, "RMSprop": FusedRMSprop}[opt_name](model.parameters(), **opt_kw)

    def step():
        opt.zero_grad()
        loss = loss_fn(model(x))
        loss.backward()
        opt.step()
        return loss

    return step, B


def build(args, device, rank=0):
    """-> (module, loss_fn(out) -> scalar, x, B, size). The optimizer is NOT built here: it is
    constructed after the data-parallel wrapper has laid the parameters out (main())."""
    import torch

    from deep_vision_amd import ops as F
    from deep_vision_amd.models import get_model

    B, size, _, _, fam = SPECS[args.model]
    B = args.batch or B
    lo = rank * B  # this rank's slice of the global synthetic batch
    if fam == "cls":
        model = get_model(args.model).to(device)
        cin = 1 if args.model == "lenet5" else 3
        ncls = 10 if args.model == "lenet5" else 1000
        smp = [_sample_cls(lo + i, cin, size, ncls) for i in range(B)]
        x = torch.stack([a for a, _ in smp]).to(device)
        y = torch.tensor([b for _, b in smp], dtype=torch.int64).to(device)
        del smp
        if args.model == "inception1":
            def loss_fn(out):  # main + 0.3 x aux heads
                if isinstance(out, tuple):
                    return F.cross_entropy(out[0], y) + 0.3 * (F.cross_entropy(out[1], y) + F.cross_entropy(out[2], y))
                return F.cross_entropy(out, y)
        elif args.backend == "torch":
            def loss_fn(out):
                return torch.nn.functional.cross_entropy(out.float(), y)
        else:
            def loss_fn(out):
                return F.cross_entropy(out, y)
    elif fam == "yolo":
        from deep_vision_amd.data import yolo as Y
        from deep_vision_amd.train.detection import yolo_loss

        model = get_model("yolov3", num_classes=80).to(device)
        ds = Y.SyntheticYoloDataset(lo + B, 80, size, 1)
        imgs, labels = Y.collate([ds[lo + i] for i in range(B)])
        x = imgs.to(device)
        lab = tuple(t.to(device) for t in labels)

        def loss_fn(out):
            return yolo_loss(out, lab, 80)[0] / B
    elif fam == "hourglass":
        from deep_vision_amd.data import pose as P
        from deep_vision_amd.train.detection import hourglass_loss

        model = get_model("hourglass104", num_stack=4, num_residual=1, num_heatmap=16).to(device)
        ds = P.SyntheticPoseDataset(lo + B, size, (size // 4, size // 4, 16), 1)
        items = [ds[lo + i] for i in range(B)]
        x = torch.stack([torch.from_numpy(a) for a, _ in items]).to(device)
        hm = torch.stack([torch.from_numpy(b) for _, b in items]).to(device)

        def loss_fn(out):
            return hourglass_loss(out, hm)[0] / B
    else:
        raise ValueError(fam)
    if args.backend == "torch" and device.type == "cuda":
        model = model.to(memory_format=torch.channels_last)
        x = x.contiguous(memory_format=torch.channels_last)
    return model, loss_fn, x, B, size


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=0, help="per-GPU batch (0 = the config's)")
    ap.add_argument("--model", default="resnet50", choices=sorted(SPECS))
    ap.add_argument("--backend", default="native", choices=["native", "torch"],
                    help="torch = PyTorch/MIOpen reference path (for comparison only)")
    ap.add_argument("--write-comparator", action="store_true",
                    help="with --backend torch: record this run as the same-box comparator of the native arm "
                         "(profiles/bench_<model>_1gpu_torch_miopen.json)")
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--comm-dtype", default="fp32", choices=["fp32", "bf16"],
                    help="gradient all-reduce wire format (fp32 master gradients either way)")
    ap.add_argument("--device", default=None, help="cpu to force the CPU plumbing path")
    ap.add_argument("--force-dp", action="store_true",
                    help="wrap in DataParallel and all-reduce over a process group even at world size 1 "
                         "(exercises the RCCL bucket path on one GPU)")
    ap.add_argument("--graph", action=argparse.BooleanOptionalAction, default=None,
                    help="capture the training step (data-parallel all-reduces included) as a HIP graph and "
                         "replay it (deep_vision_amd/train/graph.py); default: the model's measured-faster "
                         "mode (deep_vision_amd/policy.py PREFERRED)")
    ap.add_argument("--policy", action="store_true",
                    help="print this process's resolved stream / queue policy as JSON and exit (no GPU use)")
    args = ap.parse_args()
    # an explicit --graph stands; the per-model default applies to the native GPU path only
    args.graph = GRAPH and (_PRE.graph is not None or (args.backend == "native" and args.device != "cpu"))
    if args.policy:
        rec = _policy.describe()
        rec["rank"] = int(__import__("os").environ.get("RANK", "0"))
        sys.stdout.flush()
        # one write(2) per line: the ranks of a torchrun share the pipe, and a line written in pieces
        # (text + newline) could interleave with another rank's
        __import__("os").write(sys.stdout.fileno(), (json.dumps(rec) + "\n").encode())
        return

    import os

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and args.device != "cpu":
        # self-launch N ranks; this parent never initialises the GPU
        from deep_vision_amd.launch import spawn

        sys.exit(spawn(args.gpus, [os.path.abspath(__file__)] + sys.argv[1:], graph=args.graph))

    if "WORLD_SIZE" in os.environ:  # a rank: its own NUMA-local CPU set before any GPU / thread-pool use
        from deep_vision_amd.launch import pin_rank_cpus

        pin_rank_cpus()

    import threading

    def heartbeat():  # long silent phases (MIOpen kernel search of the torch arm) print to stderr
        t0 = time.time()
        while True:
            time.sleep(60)
            print(f"[bench] alive {time.time() - t0:.0f}s", file=sys.stderr, flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()

    import torch
    import torch.distributed as dist

    from deep_vision_amd import ops as F
    from deep_vision_amd.parallel.ddp import DataParallel
    from deep_vision_amd.parallel.dist import barrier, init_distributed, is_dist

    if args.graph:
        from deep_vision_amd.train.graph import prepare_capture_env

        prepare_capture_env()  # captured RCCL all-reduces (train/graph.py), before the group exists
    world, rank, local, device = init_distributed("gloo" if args.device == "cpu" else None, force=args.force_dp)
    if args.device == "cpu":
        device = torch.device("cpu")
    if world != args.gpus and args.device != "cpu":
        raise SystemExit(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a mismatched run")
    F.set_backend(args.backend)
    torch.manual_seed(1234 + rank)
    torch.backends.cudnn.benchmark = True
    cuda = device.type == "cuda"

    def sync():
        if cuda:
            torch.cuda.synchronize()

    from deep_vision_amd.train.optim import OPTIMIZERS

    model, loss_fn, x, B, size = build(args, device, rank)
    ddp = (DataParallel(model, bucket_mb=args.bucket_mb, timing=cuda, always_reduce=args.force_dp,
                        comm_dtype=torch.bfloat16 if args.comm_dtype == "bf16" else torch.float32)
           if (is_dist() or args.force_dp) else None)
    # the optimizer binds to the flat parameter buffer AFTER DataParallel laid it out (it would
    # also re-bind transparently: train.optim._FlatOptimizer._check_binding)
    _, _, opt_name, opt_kw, _ = SPECS[args.model]
    opt = OPTIMIZERS[opt_name](model.parameters(), **opt_kw)
    gscale = ddp.grad_scale if ddp else 1.0
    net = ddp if ddp else model
    amp = args.backend == "torch" and cuda

    def step():
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            out = net(x)
            loss = loss_fn(out)
        loss.backward()
        if ddp:
            ddp.finish()
        opt.step(grad_scale=gscale)
        return loss

    def global_loss(loss):
        """Mean of the per-rank losses = the loss over the global batch (equal shards)."""
        v = loss.detach().float().reshape(1).to(torch.float64)
        if is_dist():
            dist.all_reduce(v)
            v /= world
        return float(v.item())

    if args.graph:
        if not cuda or amp:
            raise SystemExit("[bench] --graph needs the native GPU path")
        from deep_vision_amd.train.graph import CapturedStep

        opt.use_device_guard(True)  # the trainers' captured step: non-finite skip decided on the device
        cap = CapturedStep(step, opt, model=model, warmup=2)  # 2 eager side-stream steps, then capture
        step = cap  # noqa: F811 - replays from here on

    # multi-rank runs: every step's GPU completion is watched (a dead / wedged peer ends the rank
    # instead of hanging the job; captured all-reduces run without RCCL's own async error handling)
    cwd = None
    if cuda and is_dist():
        from deep_vision_amd.parallel.watchdog import CommWatchdog

        cwd = CommWatchdog().start()
        inner = step

        def step():  # noqa: F811
            out = inner()
            ev = torch.cuda.Event()
            ev.record()
            cwd.track("bench step", ev)
            return out

    import contextlib

    # eager steps run on a high-priority stream of their own, so the weight-gradient side stream
    # (normal priority) soaks up the CUs the main path leaves idle instead of competing for them:
    # ResNet-50 13,936 -> 14,017 / 14,044 img/s, same box, two pairs (profiles/main_stream_priority_ab.txt).
    # DV_MAIN_PRIO=0 keeps the default stream.
    prio = contextlib.nullcontext()
    if cuda and os.environ.get("DV_MAIN_PRIO", "1") == "1" and not args.graph:
        main_stream = torch.cuda.Stream(device=device, priority=-1)
        main_stream.wait_stream(torch.cuda.current_stream(device))
        prio = torch.cuda.stream(main_stream)
    with prio:
        for _ in range(args.warmup):
            loss = step()
        sync()
        first_loss = global_loss(loss) if args.warmup else float("nan")

        barrier()
        sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            loss = step()
        sync()
        barrier()
        sync()
        dt = time.perf_counter() - t0

    if is_dist():
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    last_loss = global_loss(loss)
    ms = dt / args.steps * 1e3
    imgs = B * world * args.steps / dt
    comm_ms = ddp.exposed_comm_ms(last=args.steps) if (ddp is not None and cuda) else 0.0
    if is_dist():
        t = torch.tensor([comm_ms], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        comm_ms = float(t.item())
    if rank == 0:
        base = BASELINES.get(args.model)
        miopen, miopen_src = same_box_miopen(args.model)
        if args.model == "resnet50":
            metric = RESNET_METRIC
        else:
            metric = f"images/sec (whole node), {args.model} {size}x{size} {'bf16' if cuda else 'fp32'}"
        rec = {
            "metric": metric,
            "value": round(imgs, 2),
            "unit": "images/sec",
            "n_gpus": world if cuda else 0,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(imgs / base, 3) if base else None,
            "vs_baseline_basis": ("BASELINE.md reference proxy: images/s of a whole 8-GPU K80-era fp32 node "
                                  "(not like-for-like; see vs_same_box_miopen)") if base else None,
            "vs_same_box_miopen": (round(imgs / (miopen * world), 3)
                                   if miopen and cuda and args.backend == "native" else None),
            "vs_same_box_miopen_src": miopen_src if (miopen and cuda and args.backend == "native") else None,
            "per_gpu": round(imgs / max(1, world), 2),
            "comm_exposed_ms": round(comm_ms, 3),
            "dtype": "bf16" if cuda else "fp32",
            "data": ("synthetic (classification: 100 class templates + noise, a learnable fixed batch; "
                     "others: random inputs / labels of the config's shapes; random-init weights)"),
            "config": {
                "model": args.model,
                "global_batch": B * world,
                "per_gpu_batch": B,
                "seq_len": None,
                "image_size": size,
                "parallelism": f"dp{world}",
                "comm_dtype": args.comm_dtype,
                "bucket_mb": args.bucket_mb,
                "optimizer": f"{type(opt).__name__} {SPECS[args.model][3]}",
                "backend": args.backend,
                "hip_graph": bool(args.graph),
                "device": str(device),
                "loss_first_last": [round(first_loss, 4), round(last_loss, 4)],
            },
        }
        print(json.dumps(rec), flush=True)
        if args.backend == "torch" and cuda and world == 1 and args.steps >= 10 and args.write_comparator:
            with open(comparator_path(args.model), "w") as f:  # the measured comparator of the native arm
                f.write(json.dumps(rec) + "\n")
    if cwd is not None:
        cwd.stop()
    if dist.is_available() and dist.is_initialized():  # also the world-1 group of --force-dp
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
