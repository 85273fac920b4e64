#!/usr/bin/env python3
"""Flagship benchmark: ResNet-50 V1 bf16 training throughput (images/sec, whole job).

Config named by BASELINE.json: ResNet-50 224x224 bf16, synthetic ImageNet-shaped data,
random-init weights, SGD(lr .1, momentum .9, wd 1e-4) as R/ResNet/pytorch/train.py:166-184,
per-GPU batch 256 (weak scaling), data parallel over RCCL with one process per GPU.

Every timed step is a full training step: forward, softmax-CE loss, backward, bucketed
gradient all-reduce (N > 1), fused SGD update, gradient zeroing.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--model resnet50]
        (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# Reference-derived comparator: ResNet-50-equivalent proxy ~376 img/s per node.
BASELINE_IMG_S = 376.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--backend", default="native", choices=["native", "torch"],
                    help="torch = PyTorch/MIOpen reference path (for comparison only)")
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--profile-steps", type=int, default=0)
    args = ap.parse_args()

    import torch

    from deep_vision_amd import ops as F
    from deep_vision_amd.models import get_model
    from deep_vision_amd.parallel.ddp import DataParallel
    from deep_vision_amd.parallel.dist import barrier, init_distributed, is_dist
    from deep_vision_amd.train.optim import FusedSGD

    world, rank, local, device = init_distributed()
    if world != args.gpus and rank == 0:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    F.set_backend(args.backend)
    torch.manual_seed(1234 + rank)
    torch.backends.cudnn.benchmark = True

    model = get_model(args.model).to(device)
    if args.backend == "torch":
        model = model.to(memory_format=torch.channels_last)
    ddp = DataParallel(model, bucket_mb=args.bucket_mb) if is_dist() else None
    opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    gscale = ddp.grad_scale if ddp else 1.0
    net = ddp if ddp else model

    B = args.batch
    x = torch.randn(B, 3, 224, 224, device=device)
    if args.backend == "torch":
        x = x.to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (B,), device=device)

    def step():
        opt.zero_grad()
        if args.backend == "torch":
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = net(x)
                loss = torch.nn.functional.cross_entropy(out.float(), y)
        else:
            out = net(x)
            loss = F.cross_entropy(out, y)
        loss.backward()
        if ddp:
            ddp.finish()
        opt.step(grad_scale=gscale)
        return loss

    for _ in range(args.warmup):
        loss = step()
    torch.cuda.synchronize()
    first_loss = float(loss.item()) if args.warmup else float("nan")

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0

    if is_dist():
        import torch.distributed as dist

        t = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    last_loss = float(loss.item())
    ms = dt / args.steps * 1e3
    imgs = B * world * args.steps / dt
    if rank == 0:
        rec = {
            "metric": "images/sec (whole node), ResNet-50 224x224 bf16 at 1/2/4/8 MI355X",
            "value": round(imgs, 2),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(imgs / BASELINE_IMG_S, 3),
            "dtype": "bf16",
            "data": "synthetic (random 224x224x3 images / labels, random-init weights)",
            "config": {
                "model": args.model,
                "global_batch": B * world,
                "per_gpu_batch": B,
                "seq_len": None,
                "image_size": 224,
                "parallelism": f"dp{world}",
                "optimizer": "SGD(lr=0.1, momentum=0.9, wd=1e-4) fused",
                "backend": args.backend,
                "loss_first_last": [round(first_loss, 4), round(last_loss, 4)],
            },
        }
        print(json.dumps(rec), flush=True)
    if is_dist():
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
