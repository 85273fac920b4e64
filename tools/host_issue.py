"""Host issue time per rank of the eager training step, alone and with N processes issuing at once.

    python tools/host_issue.py [--model resnet50] [--batch 32] [--procs 1,8] [--steps 6]

Each process builds the bench step (bench.build_step_for_profile), warms up, then -- after a
gloo barrier on 127.0.0.1 so that all N issue together -- times ``--steps`` steps WITHOUT a
device sync in between: at a small batch the GPU finishes each step faster than Python issues
it, so the wall time per step is the host's issue time (kernel launches + autograd + Python). The
GPU completion time follows after the final sync. Every process pins its CPUs like a training
rank (launch.pin_rank_cpus with LOCAL_RANK / LOCAL_WORLD_SIZE = N). The parent never touches the
GPU: it starts the N children as processes and collects one JSON line from each.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(a):
    from deep_vision_amd.launch import pin_rank_cpus

    pin_rank_cpus()
    import torch
    import torch.distributed as dist

    import bench

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    step, nimg = bench.build_step_for_profile(a.model, a.batch)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    dist.barrier()
    print(json.dumps({"rank": rank, "procs": world, "issue_ms": 1e3 * (t1 - t0) / a.steps,
                      "complete_ms": 1e3 * (t2 - t0) / a.steps, "cpus": len(os.sched_getaffinity(0)),
                      "images_per_step": nimg}), flush=True)
    dist.destroy_process_group()


def parent(a):
    from deep_vision_amd.launch import free_port

    out = []
    for n in [int(v) for v in a.procs.split(",")]:
        port = free_port()
        procs = []
        for r in range(n):
            env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
            env.setdefault("OMP_NUM_THREADS", "2")
            cmd = [sys.executable, os.path.abspath(__file__), "--child", "--model", a.model, "--batch", str(a.batch),
                   "--steps", str(a.steps)]
            procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, cwd=ROOT))
        rows = []
        for p in procs:
            so, _ = p.communicate(timeout=a.timeout)
            if p.returncode != 0:
                raise SystemExit(f"child exited with {p.returncode}")
            rows += [json.loads(line) for line in so.splitlines() if line.startswith("{")]
        rows.sort(key=lambda r: r["rank"])
        iss = [r["issue_ms"] for r in rows]
        print(f"# {a.model} batch {a.batch}/process, {n} process(es) issuing together: host issue ms/step "
              f"per rank min {min(iss):.2f} / median {sorted(iss)[len(iss) // 2]:.2f} / max {max(iss):.2f}", flush=True)
        for r in rows:
            print("  " + json.dumps(r), flush=True)
        out.append(rows)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--procs", default="1,8")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--timeout", type=int, default=600)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        child(a)
    else:
        parent(a)


if __name__ == "__main__":
    main()
