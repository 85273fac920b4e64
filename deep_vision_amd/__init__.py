"""deep_vision_amd — an MI355X-native (gfx950 / CDNA4) classic-CNN vision training framework.

Capabilities of zackdilan/deep-vision (model zoo, per-model trainers, checkpoint layouts),
re-designed around hand-written HIP kernels (MFMA implicit-GEMM convolution, fused
BatchNorm, pooling, loss, optimizers) and one-process-per-GPU data parallelism over RCCL.
"""
__version__ = "0.1.0"

from . import ops  # noqa: F401,E402


def set_deterministic(on: bool = True) -> None:
    """Bitwise-reproducible weight gradients: split-K wgrad partials go through per-split slabs
    summed in a fixed order instead of fp32 atomics (also ``DV_DETERMINISTIC=1``). BatchNorm
    statistics keep their sharded atomics (order effects at the fp32 ulp level)."""
    from ._ext import lib

    lib().set_deterministic(bool(on))


def set_sync_check(on: bool = True) -> None:
    """Synchronise and check for HIP errors after every native launch (also ``DV_SYNC_CHECK=1``):
    an asynchronous GPU fault is then raised by the op that caused it."""
    from ._ext import lib

    lib().set_sync_check(bool(on))
