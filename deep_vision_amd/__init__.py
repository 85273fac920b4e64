"""deep_vision_amd — an MI355X-native (gfx950 / CDNA4) classic-CNN vision training framework.

Capabilities of zackdilan/deep-vision (model zoo, per-model trainers, checkpoint layouts),
re-designed around hand-written HIP kernels (MFMA implicit-GEMM convolution, fused
BatchNorm, pooling, loss, optimizers) and one-process-per-GPU data parallelism over RCCL.
"""
__version__ = "0.1.0"

from . import ops  # noqa: F401,E402
