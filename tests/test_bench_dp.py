"""The benchmark's own data-parallel wiring, end to end on CPU.

``bench.py --gpus 2`` under ``torch.distributed.run`` (two gloo ranks) must train exactly like one
process over the same global batch: the synthetic samples are a pure function of their global
index (bench._sample_cls), DataParallel broadcasts rank 0's initial weights, and the optimizer is
bound to the flat buffer DataParallel laid out. LeNet-5 has no BatchNorm, so the per-replica BN
statistics cannot make the two runs differ. The round-2 bench built the optimizer first: the dp2
run then kept a constant loss ([2.3041, 2.3041]) while dp1 trained.
"""
import json
import os
import subprocess
import sys

import pytest

from deep_vision_amd.launch import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(cmd):
    env = dict(os.environ, OMP_NUM_THREADS="2")
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 alone prints ONE JSON line
    return json.loads(lines[0])


@pytest.mark.timeout(900)
def test_bench_dp2_trains_like_dp1_on_global_batch():
    steps, warm = 8, 2
    one = _run([sys.executable, "bench.py", "--device", "cpu", "--model", "lenet5", "--batch", "128",
                "--steps", str(steps), "--warmup", str(warm)])
    two = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                "--master-addr=127.0.0.1", f"--master-port={free_port()}", "bench.py", "--gpus", "2",
                "--device", "cpu", "--model", "lenet5", "--steps", str(steps), "--warmup", str(warm)])
    assert two["config"]["parallelism"] == "dp2" and two["config"]["global_batch"] == 128
    assert one["config"]["global_batch"] == 128
    f1, l1 = one["config"]["loss_first_last"]
    f2, l2 = two["config"]["loss_first_last"]
    assert l1 < f1 - 0.02, (f1, l1)  # the single process trains
    assert l2 < f2 - 0.02, (f2, l2)  # ... and so does the DP run
    assert f2 == pytest.approx(f1, abs=2e-4)
    assert l2 == pytest.approx(l1, abs=2e-4)
