"""deep_vision_amd — an MI355X-native (gfx950 / CDNA4) classic-CNN vision training framework.

Capabilities of zackdilan/deep-vision (model zoo, per-model trainers, checkpoint layouts),
re-designed around hand-written HIP kernels (MFMA implicit-GEMM convolution, fused
BatchNorm, pooling, loss, optimizers) and one-process-per-GPU data parallelism over RCCL.
"""
__version__ = "0.1.0"


def __getattr__(name):
    # subpackages load on first use, so ``deep_vision_amd.policy`` can be imported (and the launch
    # environment set) before torch / HIP are touched
    if name in ("ops", "nn", "models", "train", "data", "parallel", "utils", "profiling", "inference"):
        import importlib

        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)


def set_deterministic(on: bool = True) -> None:
    """Whole-step deterministic mode (also ``DV_DETERMINISTIC=1``): the same training step run twice
    from the same state gives bitwise-equal losses, gradients and weights.

    Every cross-block accumulation of the training path stops using float atomics in arbitrary
    order: split-K / depthwise / grouped / stem weight gradients go through per-block fp32 slabs
    summed in a fixed order; BatchNorm statistics and backward sums (conv / dgrad / depthwise /
    grouped / stem / fused-pool epilogues, the separate reduction passes, bias channel sums) write
    one partial row per block into a per-stream slab that a fold kernel adds, in block order, into
    the 64 accumulator shards (csrc/kernels.h DetStats); loss totals likewise (dv_det_sum). Costs
    one extra small launch per statistics producer (profiles/deterministic_cost.txt)."""
    from ._ext import lib

    lib().set_deterministic(bool(on))


def set_sync_check(on: bool = True) -> None:
    """Synchronise and check for HIP errors after every native launch (also ``DV_SYNC_CHECK=1``):
    an asynchronous GPU fault is then raised by the op that caused it."""
    from ._ext import lib

    lib().set_sync_check(bool(on))
