"""The lazily counted ``num_batches_tracked`` (ops/bn.py _count_batch) keeps torch semantics:
in-place rewrites of the buffer (reset_running_stats, load_state_dict) replace pending steps,
copies (deepcopy) carry them, state_dict and momentum=None see the exact count.
Reference semantics: torch.nn.BatchNorm2d as used throughout R/*/pytorch (e.g.
R/ResNet/pytorch/models/resnet.py BatchNorm2d layers)."""
import copy

import torch

from deep_vision_amd.ops.bn import _count_batch, bn_momentum


def _n(bn):
    return int(bn.state_dict()["num_batches_tracked"])


def test_pending_count_flushes_on_state_dict():
    bn = torch.nn.BatchNorm2d(4)
    for _ in range(3):
        _count_batch(bn)
    assert int(bn.num_batches_tracked) == 0  # still pending on the host
    assert _n(bn) == 3
    _count_batch(bn)
    assert _n(bn) == 4


def test_reset_running_stats_voids_pending_steps():
    bn = torch.nn.BatchNorm2d(4)
    _count_batch(bn)
    _count_batch(bn)
    bn.reset_running_stats()
    assert _n(bn) == 0
    _count_batch(bn)
    assert _n(bn) == 1


def test_load_state_dict_replaces_pending_steps():
    bn = torch.nn.BatchNorm2d(4)
    sd = copy.deepcopy(bn.state_dict())
    sd["num_batches_tracked"] = torch.tensor(10)
    _count_batch(bn)
    bn.load_state_dict(sd)
    assert _n(bn) == 10
    _count_batch(bn)
    assert _n(bn) == 11


def test_deepcopy_carries_pending_steps():
    bn = torch.nn.BatchNorm2d(4)
    _count_batch(bn)
    _count_batch(bn)
    cp = copy.deepcopy(bn)
    assert _n(cp) == 2 and _n(bn) == 2
    cp.reset_running_stats()
    cp.momentum = None
    _count_batch(cp)
    assert bn_momentum(cp) == 1.0  # cumulative average restarts after a reset
    _count_batch(cp)
    assert bn_momentum(cp) == 0.5


def test_framework_batchnorm_copy_then_reset():
    """deep_vision_amd.nn.BatchNorm2d: a deepcopy flushes the pending count into the copy, and
    reset_running_stats on the copy drops everything (tools/diag_eval_gap.py's recalibration)."""
    from deep_vision_amd import nn

    bn = nn.BatchNorm2d(4)
    _count_batch(bn)
    _count_batch(bn)
    cp = copy.deepcopy(bn)
    assert int(cp.num_batches_tracked) == 2 and _n(bn) == 2
    cp.reset_running_stats()
    cp.momentum = None
    _count_batch(cp)
    assert bn_momentum(cp) == 1.0
