"""In-tree build of the native gfx950 extension ``deep_vision_amd._C``.

Every ``csrc/*.hip`` / ``csrc/*.cpp`` translation unit is compiled by ``hipcc
--offload-arch=gfx950`` into ``build/`` and linked into ``deep_vision_amd/_C*.so``.

The extension links against the HIP runtime bundled with torch (``torch/lib``) rather than
``/opt/rocm/lib`` so that a single HIP runtime lives in the process (torch ships the ROCm
7.0 runtime, the toolchain here is ROCm 7.2; both export the same soname, and loading two
would give two independent device contexts).

Usage: ``python -m deep_vision_amd._build [--force] [-j N] [--debug]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build")
PKG = os.path.join(ROOT, "deep_vision_amd")
ARCH = os.environ.get("DV_OFFLOAD_ARCH", "gfx950")


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def ext_path() -> str:
    return os.path.join(PKG, "_C" + _ext_suffix())


def _torch_lib() -> str:
    import importlib.util

    spec = importlib.util.find_spec("torch")
    if spec is None or spec.origin is None:
        raise RuntimeError("torch is required to build deep_vision_amd")
    return os.path.join(os.path.dirname(spec.origin), "lib")


def _sources():
    out = []
    for f in sorted(os.listdir(CSRC)):
        if f.endswith((".hip", ".cpp")) and os.path.isfile(os.path.join(CSRC, f)):
            out.append(os.path.join(CSRC, f))
    return out


def _headers_mtime() -> float:
    m = 0.0
    for f in os.listdir(CSRC):
        if f.endswith((".h", ".hpp")):
            m = max(m, os.path.getmtime(os.path.join(CSRC, f)))
    return m


def _compile(src: str, debug: bool) -> str:
    import pybind11

    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    flags = ["-O3"] if not debug else ["-O1", "-g"]
    cmd = [
        "hipcc", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", *flags, "-c", src, "-o", obj,
        f"-I{CSRC}", f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}",
        "-Wno-unused-result", "-Wno-unused-value",
    ]
    if debug:
        cmd.append("-DDV_DEBUG=1")
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int | None = None, debug: bool = False, verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    srcs = _sources()
    hdr_m = _headers_mtime()
    todo = []
    objs = []
    for s in srcs:
        obj = os.path.join(BUILD, os.path.basename(s) + ".o")
        objs.append(obj)
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(s), hdr_m):
            todo.append(s)
    out = ext_path()
    if todo:
        jobs = jobs or min(len(todo), max(1, (os.cpu_count() or 4) // 2), 8)
        if verbose:
            print(f"[deep_vision_amd] compiling {len(todo)} TU(s) for {ARCH} with {jobs} job(s)", flush=True)
        with cf.ThreadPoolExecutor(jobs) as ex:
            list(ex.map(lambda s: _compile(s, debug), todo))
    if todo or not os.path.exists(out) or any(os.path.getmtime(o) > os.path.getmtime(out) for o in objs):
        tl = _torch_lib()
        cmd = ["g++", "-shared", "-o", out, *objs, f"-L{tl}", "-l:libamdhip64.so", f"-Wl,-rpath,{tl}"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(f"[deep_vision_amd] linked {out}", flush=True)
    return out


def io_ext_path() -> str:
    return os.path.join(PKG, "_io" + _ext_suffix())


def build_host(force: bool = False, verbose: bool = True) -> str:
    """Host-only native runtime (csrc/host/*.cpp -> deep_vision_amd._io): g++, SSE4.2 CRC32C."""
    import pybind11

    srcs = sorted(os.path.join(CSRC, "host", f) for f in os.listdir(os.path.join(CSRC, "host")) if f.endswith(".cpp"))
    out = io_ext_path()
    deps = srcs + [os.path.join(CSRC, "host", f) for f in os.listdir(os.path.join(CSRC, "host")) if f.endswith(".h")]
    if not force and os.path.exists(out) and all(os.path.getmtime(s) <= os.path.getmtime(out) for s in deps):
        return out
    cmd = ["g++", "-O3", "-msse4.2", "-std=c++17", "-shared", "-fPIC", "-pthread", *srcs, "-o", out,
           f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"host build failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"[deep_vision_amd] built {out}", flush=True)
    return out


def build_all(force: bool = False, verbose: bool = True) -> None:
    build(force=force, verbose=verbose)
    build_host(force=force, verbose=verbose)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--debug", action="store_true")
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.j, debug=a.debug)
    build_host(force=a.force)


if __name__ == "__main__":
    sys.exit(main())
