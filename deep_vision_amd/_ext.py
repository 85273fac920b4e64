"""Loader for the native gfx950 extension.

On a GPU process the extension is mandatory: ``lib()`` raises if ``_C`` cannot be imported,
so a GPU run can never silently fall back to PyTorch kernels. CPU-only processes (unit
tests, LeNet plumbing) never touch it.
"""
from __future__ import annotations

import os

import torch  # noqa: F401  (must load torch's HIP runtime before _C)

_lib = None
_err = None


def lib():
    global _lib, _err
    if _lib is not None:
        return _lib
    try:
        from . import _C  # type: ignore

        _lib = _C
        return _lib
    except Exception as e:  # pragma: no cover - depends on build state
        _err = e
        if os.environ.get("DV_AUTOBUILD", "1") == "1":
            from . import _build

            _build.build(verbose=True)
            from . import _C  # type: ignore

            _lib = _C
            return _lib
        raise RuntimeError(
            "deep_vision_amd native extension (_C) is not built; run `python -m deep_vision_amd._build`"
        ) from e


def available() -> bool:
    try:
        lib()
        return True
    except Exception:
        return False


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_CUR_DEV = getattr(torch._C, "_cuda_getDevice", None)


def stream_handle(device=None) -> int:
    """The current HIP stream of ``device`` (default: the current device) as an integer handle.
    Called once per kernel launch: the raw-pointer query skips building a torch.cuda.Stream
    object (a few microseconds per launch on the launch-bound models)."""
    if device is None and _RAW_STREAM is not None:
        return _RAW_STREAM(_CUR_DEV())
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()
