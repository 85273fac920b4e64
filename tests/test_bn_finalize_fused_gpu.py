"""BatchNorm finalize fused into the producer conv (csrc/conv_fwd_core.h fin_tail, ops.bn
FUSE_FINALIZE): the last block of every output-column tile folds the statistics shards and writes
scale / shift / mean / invstd, the next shift row and the running statistics. Checked against the
separate bn_finalize launch on the same inputs over several steps (the shards re-zero and the
tickets reset, so step 2+ depend on both), on every tile shape of the heuristic, partial tiles
and a grouped conv; the statistics workspace must be clean after each step.
"""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"

CASES = [
    # N, C, H, W, O, k, stride, groups, fused   (tile picked by the heuristic)
    (4, 64, 28, 28, 64, 1, 1, 1, True),         # 256x64, 3-stage ring
    (16, 64, 28, 28, 128, 3, 1, 1, True),       # 128x128
    (8, 128, 23, 23, 200, 3, 1, 1, True),       # partial M and N tiles
    (16, 96, 63, 63, 64, 3, 2, 1, True),        # strided, 256x64, long K
    (4, 128, 14, 14, 128, 3, 1, 2, True),       # grouped: G = 2 column groups
    (256, 1024, 14, 14, 256, 1, 1, 1, True),    # 256x256 8-wave tile (>= 192 tiles)
    (3, 128, 7, 9, 200, 3, 1, 1, False),        # split-K grid: separate finalize (fallback)
]


def _nhwc(t):
    return t.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("case", CASES)
def test_fused_finalize_matches_separate_pass(case):
    from deep_vision_amd import nn
    from deep_vision_amd import ops as F
    from deep_vision_amd.ops import bn as B
    from deep_vision_amd.ops.common import workspace

    N, C, H, W, O, k, s, g, fused = case
    torch.manual_seed(1)
    conv = nn.Conv2d(C, O, k, stride=s, padding=k // 2, groups=g, bias=False).to(DEV)
    bn = nn.BatchNorm2d(O).to(DEV)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    mods = {v: (copy.deepcopy(conv), copy.deepcopy(bn)) for v in ("sep", "fused")}
    saved = B.FUSE_FINALIZE
    try:
        for step in range(3):
            x = _nhwc(torch.randn(N, C, H, W, device=DEV) * 1.5 + 0.3 * step)
            outs = {}
            for v, (cm, bm) in mods.items():
                B.FUSE_FINALIZE = v == "fused"
                n0 = B.COUNTERS["fwd_finalize_fused"]
                outs[v] = F.conv_bn_act(x, cm, bm, "relu")
                torch.cuda.synchronize()
                live = {t.data_ptr() for t in bm.__dict__.get("_dv_ws", {}).values()}
                assert (B.COUNTERS["fwd_finalize_fused"] - n0) == (1 if v == "fused" and fused else 0), (v, case)
                ws = workspace(bm, "bn_fwd", (B.STAT_ROWS, O), x.device)
                assert ws.data_ptr() in live, "not the BN's statistics workspace"
                assert not ws[: 2 * B.STAT_SHARDS].any(), "shards not re-zeroed"
                assert not ws[2 * B.STAT_SHARDS + 1].any(), "tickets not reset"
            a, b = outs["sep"].float(), outs["fused"].float()
            assert (a - b).abs().max().item() <= 1e-2 * a.abs().max().item(), (case, step)
            assert (a != b).float().mean().item() < 1e-3, (case, step)  # rare 1-ulp flips only
            sb, fb = mods["sep"][1], mods["fused"][1]
            torch.testing.assert_close(fb.running_mean, sb.running_mean, rtol=1e-5, atol=1e-6)
            torch.testing.assert_close(fb.running_var, sb.running_var, rtol=1e-5, atol=1e-6)
            ks = workspace(sb, "bn_fwd", (B.STAT_ROWS, O), x.device)[2 * B.STAT_SHARDS]
            kf = workspace(fb, "bn_fwd", (B.STAT_ROWS, O), x.device)[2 * B.STAT_SHARDS]
            if step:
                assert ks.abs().sum() > 0  # the shift row holds the previous batch's mean
            torch.testing.assert_close(kf, ks, rtol=1e-5, atol=1e-6)  # the next batch's shift
    finally:
        B.FUSE_FINALIZE = saved


def test_fused_finalize_batch_stats_vs_fp32():
    """The fused path's normalisation against torch fp32 BatchNorm on the same bf16 conv output."""
    from deep_vision_amd import nn
    from deep_vision_amd import ops as F
    from deep_vision_amd.ops import bn as B

    torch.manual_seed(2)
    conv = nn.Conv2d(64, 128, 3, padding=1, bias=False).to(DEV)
    bn = nn.BatchNorm2d(128).to(DEV)
    ref_bn = torch.nn.BatchNorm2d(128).to(DEV)
    x = _nhwc(torch.randn(32, 64, 20, 20, device=DEV) * 2 + 1)  # 100 tiles: no split-K
    saved, B.FUSE_FINALIZE = B.FUSE_FINALIZE, True
    n0 = B.COUNTERS["fwd_finalize_fused"]
    try:
        ys = [F.conv_bn_act(x, conv, bn, None) for _ in range(2)]
    finally:
        B.FUSE_FINALIZE = saved
    assert B.COUNTERS["fwd_finalize_fused"] - n0 == 2
    ref = []
    for _ in range(2):
        with torch.no_grad():
            yc = torch.nn.functional.conv2d(x.float(), conv.weight.bfloat16().float(), padding=1)
        ref.append(ref_bn(yc.bfloat16().float()))
    for y, yr in zip(ys, ref):
        assert ((y.float() - yr).abs().max() / yr.abs().max()).item() < 2e-2
    torch.testing.assert_close(bn.running_mean, ref_bn.running_mean, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(bn.running_var, ref_bn.running_var, rtol=1e-3, atol=1e-3)
