"""Launcher: one process per GPU (SURVEY §7.1 principle 4).

``python -m deep_vision_amd.launch --nproc 8 <script.py> [args]`` or ``--nproc N`` on any family
entry point: re-runs the command under ``torch.distributed.run`` (rendezvous on 127.0.0.1) as a
*child process* and exits with its status -- the parent never touches the GPU, so nothing is
exec'ed from a GPU-initialised process.

``visible_gpu_count()`` counts GPUs without initialising HIP (the KFD topology in sysfs, filtered
by ``ROCR/HIP/CUDA_VISIBLE_DEVICES``): the TF2-origin trainers use every visible GPU by default,
like the reference's MirroredStrategy (R/Hourglass/tensorflow/train.py:195,
R/YOLO/tensorflow/train.py:281). ``pin_rank_cpus()`` gives each local rank its own NUMA-local CPU
set before any GPU call (8 ranks issuing eager steps on one host otherwise share cores).
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def _read_props(path):
    out = {}
    try:
        with open(path) as f:
            for line in f:
                k, _, v = line.partition(" ")
                try:
                    out[k] = int(v)
                except ValueError:
                    pass
    except OSError:
        pass
    return out


def kfd_gpus(root: str = KFD_NODES):
    """Properties of the GPU nodes of the KFD topology (simd_count > 0), in the runtime's device
    order (node id); [] when there is no KFD."""
    try:
        names = sorted((n for n in os.listdir(root) if n.isdigit()), key=int)
    except OSError:
        return []
    gpus = []
    for n in names:
        p = _read_props(os.path.join(root, n, "properties"))
        if p.get("simd_count", 0) > 0:
            gpus.append(p)
    return gpus


def _visible_filter(n: int):
    """Physical indices kept by the visibility variables (applied ROCR, then HIP / CUDA)."""
    idx = list(range(n))
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is None:
            continue
        keep = []
        for tok in v.split(","):
            tok = tok.strip()
            if tok.isdigit() and int(tok) < len(idx):
                keep.append(idx[int(tok)])
        idx = keep
    return idx


def visible_gpu_count(root: str = KFD_NODES) -> int:
    """Number of GPUs this process would see, without initialising HIP (the parent of a spawn must
    stay GPU-free). Falls back to torch's count (no GPU init on this image) without a KFD."""
    gpus = kfd_gpus(root)
    if gpus:
        return len(_visible_filter(len(gpus)))
    try:
        import torch

        return torch.cuda.device_count()
    except Exception:
        return 0


def resolve_nproc(nproc, device=None) -> int:
    """``--nproc``: an explicit count, or (None / 0 / "auto") one process per visible GPU -- 1 on a
    CPU-only host or with ``--device cpu``."""
    if nproc not in (None, 0, "auto", "0"):
        return int(nproc)
    if device == "cpu":
        return 1
    return max(1, visible_gpu_count())


def _cpulist(text: str):
    cpus = set()
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        cpus.update(range(int(a), int(b or a) + 1))
    return cpus


def _gpu_numa(props, sys_root="/sys") -> int:
    """NUMA node of a KFD GPU node from its PCI address (domain, location_id = bus<<8 | devfn)."""
    loc, dom = props.get("location_id"), props.get("domain", 0)
    if loc is None:
        return -1
    bdf = f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7}"
    try:
        with open(os.path.join(sys_root, "bus/pci/devices", bdf, "numa_node")) as f:
            return int(f.read().strip())
    except (OSError, ValueError):
        return -1


def rank_cpus(local_rank: int, local_world: int, allowed=None, sys_root="/sys", kfd_root=KFD_NODES):
    """The CPU set of ``local_rank``: its GPU's NUMA node's allowed CPUs, split evenly among the
    local ranks on that node; without a topology, an even split of the allowed CPUs."""
    allowed = sorted(allowed if allowed is not None else os.sched_getaffinity(0))
    if local_world <= 1 or not allowed:
        return set(allowed)
    gpus = kfd_gpus(kfd_root)
    vis = _visible_filter(len(gpus)) if gpus else []
    numa = [_gpu_numa(gpus[i], sys_root) for i in vis][:local_world] if vis else []
    if len(numa) == local_world and all(n >= 0 for n in numa):
        node = numa[local_rank]
        try:
            with open(os.path.join(sys_root, f"devices/system/node/node{node}/cpulist")) as f:
                local = sorted(_cpulist(f.read()) & set(allowed))
        except OSError:
            local = []
        peers = [r for r in range(local_world) if numa[r] == node]
        if local and len(local) >= len(peers):
            k = peers.index(local_rank)
            per = len(local) // len(peers)
            return set(local[k * per:(k + 1) * per])
    per = max(1, len(allowed) // local_world)
    lo = (local_rank * per) % len(allowed)
    return set(allowed[lo:lo + per]) or set(allowed)


def pin_rank_cpus() -> None:
    """Pin this rank (LOCAL_RANK of LOCAL_WORLD_SIZE, set by torch.distributed.run) to its CPU set
    (rank_cpus) and size its OpenMP pool to it. Call before any GPU / thread-pool use;
    ``DV_PIN_CPUS=0`` disables."""
    if os.environ.get("DV_PIN_CPUS", "1") == "0" or not hasattr(os, "sched_setaffinity"):
        return
    lw = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    if lw <= 1:
        return
    lr = int(os.environ.get("LOCAL_RANK", "0"))
    try:
        cpus = rank_cpus(lr, lw)
        if cpus:
            os.sched_setaffinity(0, cpus)
            n = min(len(cpus), int(os.environ.get("OMP_NUM_THREADS", len(cpus))))
            os.environ["OMP_NUM_THREADS"] = str(n)
            if "torch" in sys.modules:
                sys.modules["torch"].set_num_threads(n)
    except OSError:
        pass


def hw_queues_env(env, graph: bool) -> None:
    """A child environment's hardware-queue count for a step mode (deep_vision_amd/policy.py)."""
    from . import policy

    policy.queues_env(env, graph)


def spawn(nproc: int, argv, module: str | None = None, graph: bool = False) -> int:
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}"]
    cmd += (["-m", module] if module else []) + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    hw_queues_env(env, graph)
    return subprocess.call(cmd, env=env)


def maybe_spawn(nproc, device=None, graph: bool | None = None, model: str | None = None) -> bool:
    """Called first thing by the entry points, before HIP initialises. Resolves the process's step
    mode and queue policy (policy.configure: ``graph`` None -> ``model``'s measured-faster mode) and
    returns the graph decision. With ``--nproc N > 1`` (or the default: every visible GPU,
    resolve_nproc) outside a torchrun world, re-launches this script N times and exits. Inside a
    world (this script started by torchrun, ours or an external one), pins this rank's CPUs."""
    from . import policy

    graph = policy.configure(model, graph)
    if "WORLD_SIZE" in os.environ:
        pin_rank_cpus()
        return graph
    nproc = resolve_nproc(nproc, device)
    if nproc <= 1:
        return graph
    argv = list(sys.argv)
    # drop the --nproc flag so the children do not spawn again
    out, skip = [], False
    for a in argv:
        if skip:
            skip = False
            continue
        if a == "--nproc":
            skip = True
            continue
        if a.startswith("--nproc="):
            continue
        out.append(a)
    sys.exit(spawn(nproc, out, graph=graph))


def main(argv=None):
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--nproc", type=int, required=True)
    ap.add_argument("-m", "--module", default=None)
    ap.add_argument("rest", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    sys.exit(spawn(a.nproc, a.rest, a.module))


if __name__ == "__main__":
    main()
