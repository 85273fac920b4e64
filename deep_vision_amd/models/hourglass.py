"""Stacked Hourglass network (R/Hourglass/tensorflow/hourglass104.py:19-159).

* BottleneckBlock: pre-activation BN(momentum .9 -> torch .1, eps 1e-3) -> ReLU -> 1x1 (C/2) ->
  BN -> ReLU -> 3x3 (C/2) -> BN -> ReLU -> 1x1 (C), all convs with bias (Keras default), plus an
  identity or 1x1 projection (``downsample``) (:19-67).
* HourglassModule: recursive order-4 module with 2x2 max-pool down and nearest 2x up (:70-98).
* StackedHourglassNetwork: 7x7/2 stem, 4 stacks, 16 heatmaps per stack; every stack output is
  returned (intermediate supervision) and re-injected through two 1x1 convs (:101-159).

The reference's loop variable ``i`` is shadowed by the inner residual loop (:136/:138), so its
Keras graph also creates re-injection convs after the last stack. They reach no output, and a
Keras functional Model only holds layers on an input->output path, so they are not part of the
reference model and are not built here: 16,290,752 trainable parameters (pinned in tests).
SURVEY §2.2 lists 16,360,896, which counts those two dead convs (+70,144); the CenterNet
notebook summary (R/ObjectsAsPoints/tensorflow/test.ipynb cell 2) confirms that dead branches
are excluded -- models/centernet.py matches it exactly only without its dead layers.

GPU path: the BN -> ReLU prologue of each block runs as one native BN pass (statistics from a
separate reduction because the block input is a sum), the inner conv -> BN -> ReLU pairs take
their statistics from the conv epilogue.

Branch concurrency: an hourglass level's two branches (``up1`` at the level's resolution, the
pool -> low1 -> inner level -> low3 path below it) are independent until the upsample-add. At
batch 32 the 4x4 - 32x32 levels run kernels that fill a fraction of the 256 CUs, so ``up1`` runs
on a side HIP stream (one per recursion depth) forked from and joined back to the current one;
autograd runs each op's backward on its forward stream, so the backward branches overlap too, and
a captured step (train/graph.py) records the fork/join as parallel graph branches.
``BRANCH_STREAMS``: ``"graph"`` (default) forks only while a HIP graph is being captured -- an
eager step at this batch is bound by the host issuing ~1,500 launches, and the per-level
fork/join bookkeeping costs more host time than the overlap returns (measured: graph 1,024 ->
1,354 img/s, eager 631 -> 562 img/s with forking always on); ``True`` always forks; ``False``
never does. Env ``DV_BRANCH_STREAMS`` = graph / 1 / 0.
"""
from __future__ import annotations

import torch
import torch.nn as tnn

from .. import nn
from .. import ops as F
from ..ops.bn import STAT_ROWS, STAT_SHARDS
from ..ops.common import workspace
from ..ops.conv import ColsumBox, GradJoin, no_wgrad_side
from .branch import BranchEdge as _BranchEdge


import os

BRANCH_STREAMS = {"1": True, "0": False}.get(os.environ.get("DV_BRANCH_STREAMS", "graph"), "graph")
# Side streams: one per recursion depth, or -- when RCCL is active (a process group of > 1 rank) --
# two shared by depth parity (depth % side_streams()), so that with the main / capture stream and
# RCCL's own stream the process stays within GPU_MAX_HW_QUEUES = 4 hardware queues (streams beyond
# that share queues and serialise: an all-reduce could queue behind branch compute). Nested levels
# of one parity then share a stream (a level joins after the outer level's up1 too), each still
# overlapping the main stream's low branch. DV_BRANCH_SIDE_STREAMS overrides.
SIDE_STREAMS = int(os.environ.get("DV_BRANCH_SIDE_STREAMS", "0"))
_STREAMS = {}


def side_streams() -> int:
    if SIDE_STREAMS > 0:
        return SIDE_STREAMS
    import torch.distributed as dist

    multi = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    return 2 if multi else 4
_FORKED = set()  # recursion depths whose up1 branch was forked (tests)
HANDOFF_STATS = True  # a block's conv3 epilogue accumulates the next block's pre-activation BN statistics
LEVEL_JOIN = True  # an hourglass level input's three gradients are summed in one BN backward pass
BIAS_COLSUM = True  # conv3's bias gradient from the next block's BN1 backward apply pass


def _fork(x):
    if BRANCH_STREAMS is False or not F.native(x):
        return False
    if BRANCH_STREAMS == "graph":
        from ..train.graph import capturing_or_warming

        return capturing_or_warming()  # the warm-up steps fork too: they size the side streams' scratch
    return True


def _side_stream(device, depth):
    import torch

    _FORKED.add(depth)
    key = (str(device), depth % side_streams())
    st = _STREAMS.get(key)
    if st is None:
        st = _STREAMS[key] = torch.cuda.Stream(device=device)
    return st


def _bn(c):
    return nn.BatchNorm2d(c, eps=1e-3, momentum=0.1)


class BottleneckBlock(tnn.Module):
    def __init__(self, cin, filters, downsample=False):
        super().__init__()
        self.downsample = nn.Conv2d(cin, filters, 1) if downsample else None
        self.bn1 = _bn(cin)
        self.conv1 = nn.Conv2d(cin, filters // 2, 1)
        self.bn2 = _bn(filters // 2)
        self.conv2 = nn.Conv2d(filters // 2, filters // 2, 3, padding=1)
        self.bn3 = _bn(filters // 2)
        self.conv3 = nn.Conv2d(filters // 2, filters, 1)

    def forward(self, x, next_bn=None, join=None):
        # identity blocks: x's two gradients (the residual path's dy and BN1's dx) meet in BN1's
        # backward apply pass (GradJoin) instead of an autograd add -- 73 add passes per step.
        # ``join``: the hourglass level's (its pooled branch stashes a third gradient of x there)
        j = (join or GradJoin()) if self.downsample is None and F.native(x) else None
        identity = self.downsample(x) if self.downsample is not None else x
        stats, box = _take_block_stats(self.bn1, x)
        y = F.batch_norm_act(x, self.bn1, "relu", input_join=j, stats=stats, colsum=box)
        y = F.conv_bn_act(y, self.conv1, self.bn2, "relu")
        y = F.conv_bn_act(y, self.conv2, self.bn3, "relu")
        # the residual add rides in conv3's store epilogue (ops.conv2d residual=); when the next
        # block's pre-activation BN is known, the same epilogue accumulates that BN's batch
        # statistics of the block output (no separate statistics pass over it)
        if HANDOFF_STATS and next_bn is not None and next_bn.training and F.native(y):
            C = self.conv3.out_channels
            sbuf = workspace(next_bn, "bn_fwd", (STAT_ROWS, C), y.device)
            # ... and the next block's BN1 backward sums this conv's output gradient for its bias
            box = (ColsumBox(workspace(next_bn, "bias_colsum", (STAT_ROWS, C), y.device))
                   if BIAS_COLSUM and self.conv3.bias is not None else None)
            out, st = F.conv2d(y, self.conv3.weight, self.conv3.bias, residual=identity, residual_join=j,
                               want_stats=True, stats_buf=sbuf, bias_colsum=box)
            if st is not None:
                next_bn.__dict__["_dv_block_stats"] = (out.data_ptr(), out._version, tuple(out.shape), st, box)
            return out
        return F.conv2d(y, self.conv3.weight, self.conv3.bias, residual=identity, residual_join=j)


def _take_block_stats(bn, x):
    """(statistics, bias-colsum box) a producing block's conv3 handed ``bn`` -- if they are of
    exactly ``x``; otherwise the statistics shards are cleared (the workspace must be clean for the
    statistics pass the BN then runs itself) and the conv reduces its own bias gradient."""
    pre = bn.__dict__.pop("_dv_block_stats", None)
    if pre is None:
        return None, None
    if pre[:3] == (x.data_ptr(), x._version, tuple(x.shape)):
        return pre[3], pre[4]
    pre[3][: 2 * STAT_SHARDS].zero_()
    return None, None


def _entry_bn(m):
    """The pre-activation BN that first reads the input of ``m`` (a block, a block sequence or
    an hourglass level, whose input feeds its up1 branch), or None."""
    if isinstance(m, BottleneckBlock):
        return m.bn1
    if isinstance(m, tnn.Sequential) and len(m) and isinstance(m[0], BottleneckBlock):
        return m[0].bn1
    if isinstance(m, HourglassModule):
        return _entry_bn(m.up1)
    return None


def _run_blocks(blocks, x, next_bn=None, join=None):
    """A block sequence, each block handing the next one's BN statistics over (see
    BottleneckBlock.forward); the last block hands over to ``next_bn``. ``join``: the first
    block's input gradient join (HourglassModule.forward)."""
    n = len(blocks)
    for i, b in enumerate(blocks):
        x = b(x, next_bn=blocks[i + 1].bn1 if i + 1 < n else next_bn, join=join if i == 0 else None)
    return x


class HourglassModule(tnn.Module):
    def __init__(self, order, filters, num_residual):
        super().__init__()
        self.order = order
        self.up1 = tnn.Sequential(*[BottleneckBlock(filters, filters) for _ in range(num_residual + 1)])
        self.low1 = tnn.Sequential(*[BottleneckBlock(filters, filters) for _ in range(num_residual)])
        if order > 1:
            self.low2 = HourglassModule(order - 1, filters, num_residual)
        else:
            self.low2 = tnn.Sequential(*[BottleneckBlock(filters, filters) for _ in range(num_residual)])
        self.low3 = tnn.Sequential(*[BottleneckBlock(filters, filters) for _ in range(num_residual)])

    def _low(self, x, join=None):
        low = _run_blocks(self.low1, _pool(x, join, self.low1[0].bn1), next_bn=_entry_bn(self.low2))
        if isinstance(self.low2, HourglassModule):
            low = self.low2(low, next_bn=self.low3[0].bn1)
        else:
            low = _run_blocks(self.low2, low, next_bn=self.low3[0].bn1)
        return _run_blocks(self.low3, low)

    def forward(self, x, next_bn=None):
        # next_bn: the BN that reads this level's output (its statistics come from the merge pass)
        # x's gradients from up1 (block 0's BN1 and identity shortcut) and from the pool of the low
        # branch all meet in block 0's BN1 backward apply pass: no autograd add at the level input
        j = GradJoin() if LEVEL_JOIN and F.native(x) and self.up1[0].downsample is None else None
        if _fork(x):
            main = torch.cuda.current_stream(x.device)
            side = _side_stream(x.device, self.order)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                up1 = _BranchEdge.apply(_run_blocks(self.up1, _BranchEdge.apply(x, main), join=j), main)
            low = self._low(x, j)
            main.wait_stream(side)
            x.record_stream(side)  # caching allocator: x is read on the side stream
            up1.record_stream(main)
            return _merge(low, up1, next_bn)
        up1 = _run_blocks(self.up1, x, join=j)
        return _merge(self._low(x, j), up1, next_bn)


def _handoff(bn, like):
    """bn's statistics workspace when a producer pass can accumulate them (bn trains, native path)."""
    if HANDOFF_STATS and bn is not None and bn.training and F.native(like):
        return workspace(bn, "bn_fwd", (STAT_ROWS, like.shape[1]), like.device)
    return None


def _hand_over(bn, y, st):
    if st is not None:
        bn.__dict__["_dv_block_stats"] = (y.data_ptr(), y._version, tuple(y.shape), st, None)
    return y


def _pool(x, join, bn):
    """2x2 max pool of a level input; the pass also accumulates the statistics of the first low1
    block's pre-activation BN (csrc/pool.hip maxpool_fwd stats) -- no separate statistics pass."""
    sbuf = _handoff(bn, x)
    if sbuf is None:
        return F.max_pool2d(x, 2, 2, input_join=join)
    return _hand_over(bn, *F.max_pool2d(x, 2, 2, input_join=join, stats_buf=sbuf))


def _merge(low, up1, next_bn):
    """The level merge upsample(low) + up1, accumulating next_bn's statistics when known."""
    sbuf = _handoff(next_bn, up1)
    if sbuf is None:
        return F.upsample_add(low, up1, 2)
    return _hand_over(next_bn, *F.upsample_add(low, up1, 2, stats_buf=sbuf))


class StackedHourglassNetwork(tnn.Module):
    def __init__(self, num_stack=4, num_residual=1, num_heatmap=16, input_size=256):
        super().__init__()
        self.num_stack = num_stack
        self.input_size = input_size
        self.stem = nn.Conv2d(3, 64, 7, stride=2, padding="same_keras")
        self.stem_bn = _bn(64)
        self.pre = tnn.Sequential(BottleneckBlock(64, 128, downsample=True))
        self.pre2 = tnn.Sequential(BottleneckBlock(128, 128), BottleneckBlock(128, 256, downsample=True))
        self.hourglass = tnn.ModuleList(HourglassModule(4, 256, num_residual) for _ in range(num_stack))
        self.residual = tnn.ModuleList(tnn.Sequential(*[BottleneckBlock(256, 256) for _ in range(num_residual)])
                                       for _ in range(num_stack))
        self.linear = tnn.ModuleList(tnn.ModuleDict({"conv": nn.Conv2d(256, 256, 1), "bn": _bn(256)})
                                     for _ in range(num_stack))
        self.heatmap = tnn.ModuleList(nn.Conv2d(256, num_heatmap, 1) for _ in range(num_stack))
        self.inter_x = tnn.ModuleList(nn.Conv2d(256, 256, 1) for _ in range(num_stack - 1))
        self.inter_y = tnn.ModuleList(nn.Conv2d(num_heatmap, 256, 1) for _ in range(num_stack - 1))

    def forward(self, x):
        # weight gradients stay on their origin streams: a captured step forks its own branch streams
        # (a fifth stream shared their hardware queues: 1,428 -> 1,233 img/s), and the eager step is
        # host-bound (each side-stream launch adds event records / waits on the host: 913 / 771 vs
        # 682 / 770 img/s, profiles/wgrad_side_stream_ab.txt)
        with no_wgrad_side():
            return self._forward(x)

    def _forward(self, x):
        x = F.conv_bn_act(x, self.stem, self.stem_bn, "relu")
        x = _run_blocks(self.pre, x)
        x = _pool(x, None, self.pre2[0].bn1)
        x = _run_blocks(self.pre2, x, next_bn=_entry_bn(self.hourglass[0]))
        ys = []
        for i in range(self.num_stack):
            x = _run_blocks(self.residual[i], self.hourglass[i](x, next_bn=self.residual[i][0].bn1))
            lin = self.linear[i]
            x = F.conv_bn_act(x, lin["conv"], lin["bn"], "relu")
            # x feeds the heatmap conv and (but for the last stack) the re-injection conv: the
            # latter's input gradient is summed in the heatmap conv's dgrad epilogue (GradJoin)
            j = GradJoin() if i < self.num_stack - 1 and F.native(x) else None
            hm = self.heatmap[i]
            y = F.conv2d(x, hm.weight, hm.bias, join=j, join_role="consumer") if j is not None else hm(x)
            ys.append(y)
            if i < self.num_stack - 1:
                ix = self.inter_x[i]
                xi = F.conv2d(x, ix.weight, ix.bias, join=j, join_role="producer") if j is not None else ix(x)
                x = F.add(xi, self.inter_y[i](y))
        return ys
