"""Launcher helpers (deep_vision_amd/launch.py): GPU counting without initialising HIP (KFD
topology + visibility variables), one process per visible GPU by default, NUMA-local CPU sets per
local rank; and the TF2-origin entry points' all-GPU / data-parallel argument path on the CPU."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _fake_kfd(tmp_path, numa=(0, 0, 1, 1)):
    kfd = tmp_path / "kfd"
    sysr = tmp_path / "sys"
    (kfd / "0").mkdir(parents=True)
    (kfd / "0" / "properties").write_text("cpu_cores_count 64\nsimd_count 0\n")
    for i, n in enumerate(numa):
        d = kfd / str(i + 1)
        d.mkdir()
        loc = (0x10 * (i + 1)) << 8  # bus 0x10*(i+1), devfn 0
        d.joinpath("properties").write_text(f"simd_count 1024\nlocation_id {loc}\ndomain 0\n")
        bdf = f"0000:{0x10 * (i + 1):02x}:00.0"
        p = sysr / "bus" / "pci" / "devices" / bdf
        p.mkdir(parents=True)
        (p / "numa_node").write_text(f"{n}\n")
    for node, cpus in ((0, "0-15"), (1, "16-31")):
        p = sysr / "devices" / "system" / "node" / f"node{node}"
        p.mkdir(parents=True)
        (p / "cpulist").write_text(cpus + "\n")
    return str(kfd), str(sysr)


def test_visible_gpu_count_from_kfd(tmp_path, monkeypatch):
    from deep_vision_amd import launch as L

    kfd, _ = _fake_kfd(tmp_path)
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    assert L.visible_gpu_count(kfd) == 4
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1,3")
    assert L.visible_gpu_count(kfd) == 2
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "0,1,2")
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "2")
    assert L.visible_gpu_count(kfd) == 1


def test_resolve_nproc(monkeypatch):
    from deep_vision_amd import launch as L

    monkeypatch.setattr(L, "visible_gpu_count", lambda root=L.KFD_NODES: 8)
    assert L.resolve_nproc(None) == 8 and L.resolve_nproc("auto") == 8 and L.resolve_nproc(3) == 3
    assert L.resolve_nproc(None, device="cpu") == 1
    monkeypatch.setattr(L, "visible_gpu_count", lambda root=L.KFD_NODES: 0)
    assert L.resolve_nproc(None) == 1


def test_rank_cpus_numa_split(tmp_path, monkeypatch):
    from deep_vision_amd import launch as L

    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    kfd, sysr = _fake_kfd(tmp_path)
    allowed = set(range(32))
    sets = [L.rank_cpus(r, 4, allowed, sys_root=sysr, kfd_root=kfd) for r in range(4)]
    assert sets[0] == set(range(0, 8)) and sets[1] == set(range(8, 16))  # GPUs 0, 1 on NUMA node 0
    assert sets[2] == set(range(16, 24)) and sets[3] == set(range(24, 32))
    # no topology: an even split of the allowed CPUs, disjoint
    flat = [L.rank_cpus(r, 4, allowed, sys_root=str(tmp_path / "none"), kfd_root=str(tmp_path / "none"))
            for r in range(4)]
    assert all(len(s) == 8 for s in flat) and len(set().union(*flat)) == 32


def test_yolo_entry_point_two_ranks_cpu(tmp_path):
    """YOLO/tensorflow/train.py --nproc 2 spawns two gloo ranks that each run 2 steps of the
    detection engine (MirroredStrategy-style data parallelism, R/YOLO/tensorflow/train.py:281-294)."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "YOLO/tensorflow/train.py"), "--nproc", "2", "--device",
                        "cpu", "--synthetic", "--synthetic-size", "4", "--epochs", "1", "--max-steps", "2",
                        "--val-steps", "1", "--batch-size", "1", "--input-size", "64", "--workers", "0",
                        "--checkpoint-dir", str(tmp_path)], capture_output=True, text=True, cwd=str(tmp_path), env=env,
                       timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert "Using 2 ranks" in r.stdout + r.stderr


def test_hourglass_main_cli_cpu(tmp_path):
    """Hourglass/tensorflow/main.py takes --nproc / --graph (all GPUs + graph replay by default);
    on the CPU it runs one eager rank."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="4")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "Hourglass/tensorflow/main.py"), "--synthetic", "--device",
                        "cpu", "--epochs", "1", "--max_steps", "2", "--batch_size", "2", "--num_heatmap", "16",
                        "--input_size", "64", "--num_stack", "2", "--tensorboard_dir", str(tmp_path / "tb")],
                       capture_output=True, text=True, cwd=str(tmp_path), env=env, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert "Received model" in r.stdout
    r = subprocess.run([sys.executable, os.path.join(ROOT, "Hourglass/tensorflow/main.py"), "--help"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert "--nproc" in r.stdout and "--graph / --no-graph" in r.stdout


def test_hw_queue_budget_eager_vs_captured():
    """Eager ranks get 8 hardware queues (weight-gradient side stream beside RCCL's); captured steps
    keep HIP's default 4 (no side stream in a graph; Hourglass's captured branches replay faster)."""
    from deep_vision_amd.launch import hw_queues_env

    for start in ({}, {"GPU_MAX_HW_QUEUES": "4"}):
        env = dict(start)
        hw_queues_env(env, graph=False)
        assert env["GPU_MAX_HW_QUEUES"] == "8"
        env = dict(start)
        hw_queues_env(env, graph=True)
        assert env.get("GPU_MAX_HW_QUEUES", "4") == "4"
    env = {"GPU_MAX_HW_QUEUES": "16"}
    hw_queues_env(env, graph=False)
    assert env["GPU_MAX_HW_QUEUES"] == "16"
    env = {"GPU_MAX_HW_QUEUES": "4", "DV_KEEP_HW_QUEUES": "1"}
    hw_queues_env(env, graph=False)
    assert env["GPU_MAX_HW_QUEUES"] == "4"
