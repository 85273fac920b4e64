"""Merge a native and a PyTorch/MIOpen bench.py log of one model into profiles/bench_<model>_1gpu.json.

usage: python tools/zoo_profile.py <model> [gpurun_out dir] [profiles dir]
Reads gpurun_out/bench_<model>.log and gpurun_out/bench_<model>_torch.log (the JSON line of each)."""
import json
import os
import sys


def last_json(path):
    if not os.path.isfile(path):
        return None
    lines = [ln for ln in open(path) if ln.startswith("{")]
    return json.loads(lines[-1]) if lines else None


def main():
    m = sys.argv[1]
    src = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out"
    dst = sys.argv[3] if len(sys.argv) > 3 else "profiles"
    nat, ref = last_json(f"{src}/bench_{m}.log"), last_json(f"{src}/bench_{m}_torch.log")
    rec = {"model": m, "native": nat, "torch_miopen": ref,
           "speedup_vs_miopen": round(nat["value"] / ref["value"], 3) if nat and ref else None,
           "note": "1x MI355X, bench.py --steps 20 --warmup 5; torch arm = PyTorch-ROCm eager under bf16 "
                   "autocast, channels_last, cudnn.benchmark (MIOpen find)" + ("" if ref else
                                                                                "; torch arm did not finish")}
    with open(f"{dst}/bench_{m}_1gpu.json", "w") as f:
        json.dump(rec, f, indent=1)
    print(m, nat and nat["value"], ref and ref["value"], rec["speedup_vs_miopen"])


if __name__ == "__main__":
    main()
