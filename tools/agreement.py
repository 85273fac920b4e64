"""Early-step agreement of the native training step (deterministic mode) with PyTorch autocast-bf16,
from one initialisation, over several regimes and seeds. Prints per-step relative loss differences
|native - torch| / torch, the run-to-run reproducibility of the native arm, and the final losses,
so the GPU convergence tests' bounds (tests/test_convergence_gpu.py) are set from measured spreads.

usage: python tools/agreement.py [steps] [out.json]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from convergence import run as stream_run  # noqa: E402
from loss_curve import run_curve  # noqa: E402

REGIMES = [  # name, batch, lr, noise
    ("resnet50", 64, 0.01, 0.3),
    ("resnet50", 64, 0.02, 1.0),
    ("mobilenet1", 64, 0.02, 0.3),
]


def rel(a, b):
    return [round(abs(x - y) / max(abs(y), 1e-3), 4) for x, y in zip(a, b)]


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    out = {}
    for name, bs, lr, noise in REGIMES:
        for seed in (0, 1, 2):
            c = run_curve(name, bs=bs, steps=steps, lr=lr, task="learnable", noise=noise, seed=seed,
                          deterministic=True)
            c2 = run_curve(name, bs=bs, steps=steps, lr=lr, task="learnable", noise=noise, seed=seed,
                           deterministic=True, arms=("native",))
            key = f"{name} lr{lr} noise{noise} seed{seed}"
            r = rel(c["native"], c["torch-bf16"])
            out[key] = {"native": c["native"], "torch-bf16": c["torch-bf16"], "rel": r,
                        "repro": c["native"] == c2["native"]}
            print(f"{key}: repro {c['native'] == c2['native']} maxrel@5 {max(r[:5]):.4f} @10 {max(r[:10]):.4f} "
                  f"@20 {max(r[:20]):.4f} | nat {c['native'][::5]} | ref {c['torch-bf16'][::5]}", flush=True)
    for seed in (0, 1):
        r = stream_run("resnet50", bs=128, steps=steps, lr=0.1, seed=seed, every=steps, n_eval=128,
                       log=lambda s: None, deterministic=True)
        nat, ref = r["native"]["loss"], r["torch-bf16"]["loss"]
        d = rel(nat, ref)
        key = f"stream resnet50 lr0.1 seed{seed}"
        out[key] = {"native": nat, "torch-bf16": ref, "rel": d}
        print(f"{key}: maxrel@5 {max(d[:5]):.4f} @10 {max(d[:10]):.4f} @20 {max(d[:20]):.4f} | nat {nat[::5]} | "
              f"ref {ref[::5]}", flush=True)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(out, f)


if __name__ == "__main__":
    main()
