"""Process-group bootstrap: one process per GPU, RCCL (``backend="nccl"`` on ROCm) over xGMI.

Replaces the reference's single-process ``nn.DataParallel`` (R/ResNet/pytorch/train.py:353-355)
and TF ``MirroredStrategy`` (R/YOLO/tensorflow/train.py:281). Reads the torchrun environment
(RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT); CPU runs use gloo.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist


def env_world():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def init_distributed(backend: str | None = None, timeout_s: int = 600, force: bool = False):
    """Initialise the default process group if WORLD_SIZE > 1 (or always with ``force``: a world-1
    group, e.g. to exercise the RCCL path on one GPU). Returns (world, rank, local_rank, device)."""
    world, rank, local = env_world()
    backend = backend or os.environ.get("DV_DIST_BACKEND") or None
    use_cuda = torch.cuda.is_available() and (backend != "gloo" or os.environ.get("DV_DIST_BACKEND") == "gloo")
    # ranks beyond the visible device count share devices (rehearsing N ranks on fewer GPUs with
    # DV_DIST_BACKEND=gloo; RCCL itself requires one rank per GPU)
    device = torch.device(f"cuda:{local % max(1, torch.cuda.device_count())}") if use_cuda else torch.device("cpu")
    if use_cuda:
        torch.cuda.set_device(device)
    if (world > 1 or force) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1 and "MASTER_PORT" not in os.environ:
            from ..launch import free_port

            os.environ["MASTER_PORT"] = str(free_port())
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        be = backend or ("nccl" if use_cuda else "gloo")
        kw = dict(backend=be, timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kw["device_id"] = device
            # RCCL kernels on a high-priority HIP stream: the bucket all-reduces overlap a
            # backward pass that keeps every CU busy, and win the dispatch arbitration against
            # it. DV_COMM_PRIORITY=0 reverts to a normal-priority stream.
            if os.environ.get("DV_COMM_PRIORITY", "1") != "0":
                opts = dist.ProcessGroupNCCL.Options()
                opts.is_high_priority_stream = True
                kw["pg_options"] = opts
        dist.init_process_group(**kw)
    return world, rank, local, device


def is_dist():
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def world_size():
    return dist.get_world_size() if is_dist() else 1


def rank():
    return dist.get_rank() if is_dist() else 0


def barrier():
    if is_dist():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def all_reduce_scalars(values, op="sum", device=None):
    """Pack python floats into one tensor and all-reduce them in a single collective (C6/C7)."""
    t = torch.tensor(values, dtype=torch.float64, device=device or ("cuda" if torch.cuda.is_available() else "cpu"))
    if is_dist():
        dist.all_reduce(t, op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX)
    return t.tolist()


def destroy():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
