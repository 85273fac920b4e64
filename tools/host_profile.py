"""Host-side (Python) profile of eager training steps: where the launch-bound models spend the
CPU time that issues their kernels.

python tools/host_profile.py [--model hourglass] [--steps 5] [--top 40]
Runs ``--warmup`` untimed steps, then ``--steps`` steps under cProfile (GPU synchronised at the
end only, as in bench.py), and prints the functions by own time and by cumulative time.
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _instrument():
    """Wrap forward/backward of every autograd.Function in deep_vision_amd.ops with a wall-clock
    accumulator (the backward ones run on the autograd device thread, invisible to cProfile)."""
    import importlib
    import pkgutil

    import deep_vision_amd.ops as ops

    times = {}
    for mi in pkgutil.iter_modules(ops.__path__):
        mod = importlib.import_module(f"deep_vision_amd.ops.{mi.name}")
        for name, obj in list(vars(mod).items()):
            if isinstance(obj, type) and issubclass(obj, torch.autograd.Function) and obj.__module__ == mod.__name__:
                for ph in ("forward", "backward"):
                    fn = obj.__dict__.get(ph)
                    if not isinstance(fn, staticmethod):
                        continue
                    f = fn.__func__

                    def wrap(*args, _f=f, _k=(name, ph), **kw):
                        t0 = time.perf_counter()
                        try:
                            return _f(*args, **kw)
                        finally:
                            e = times.setdefault(_k, [0, 0.0])
                            e[0] += 1
                            e[1] += time.perf_counter() - t0

                    setattr(obj, ph, staticmethod(wrap))
    return times


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="hourglass")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    import bench

    step, nimg = bench.build_step_for_profile(a.model)
    times = _instrument()
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    times.clear()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(a.steps):
        step()
    pr.disable()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"# {a.model}: host issue {1e3 * (t1 - t0) / a.steps:.1f} ms/step under cProfile, "
          f"{1e3 * (t2 - t0) / a.steps:.1f} ms/step to GPU completion ({nimg} images/step)")
    print("# host time per autograd.Function (own forward / backward incl. launches), ms per step")
    for (cls, ph), (n, t) in sorted(times.items(), key=lambda kv: -kv[1][1]):
        if t * 1e3 / a.steps > 0.05:
            print(f"  {cls:28s} {ph:8s} calls/step {n / a.steps:7.1f}  {1e3 * t / a.steps:7.2f} ms  "
                  f"{1e6 * t / max(n, 1):6.1f} us/call")
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(a.top)
    st.sort_stats("cumulative").print_stats(a.top)


if __name__ == "__main__":
    main()
