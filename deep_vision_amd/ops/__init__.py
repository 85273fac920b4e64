"""Functional API of deep_vision_amd.

On CUDA (ROCm) tensors every op runs a hand-written gfx950 HIP kernel from ``csrc/``;
on CPU tensors the same call runs the PyTorch reference op (numerics oracle / CPU plumbing).
"""
from .act import activation, add, dropout, leaky_relu, relu  # noqa: F401
from .bn import batch_norm_act, batch_norm_act_maxpool, conv_bn_act, conv_bn_act_maxpool, conv_bn_deferred  # noqa: F401
from .common import as_nhwc, backend, native, set_backend  # noqa: F401
from .concat import channel_shuffle, concat, concat_slices, slice_cat  # noqa: F401
from .conv import conv2d, conv_transpose2d, linear  # noqa: F401
from .loss import cross_entropy  # noqa: F401
from .pool import adaptive_avg_pool2d, avg_pool2d, max_pool2d, upsample_add, upsample_nearest  # noqa: F401
