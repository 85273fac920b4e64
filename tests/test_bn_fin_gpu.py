"""Small BatchNorms with the statistics fold inside the apply passes (csrc/bn.hip "Small BatchNorms",
ops/bn.py FUSE_FINALIZE): against the two-launch form (bn_finalize + bn_apply, bn_bwd_finalize +
bn_bwd_apply) over several steps -- the fold order is the finalize kernel's, so outputs, input and
affine gradients, running statistics and the carried shift row are bitwise equal -- and against
a plain fp32 torch BatchNorm."""
import pytest
import torch
import torch.nn.functional as TF

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _nhwc(t):
    return t.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("C,HW,act,res", [(64, 8, "relu", False), (256, 16, "relu", True), (128, 4, None, False),
                                          (192, 13, "leaky", True), (128, 8, "leaky", "post")])
def test_fused_finalize_matches_two_launch(C, HW, act, res):
    from deep_vision_amd import nn
    from deep_vision_amd import ops as F
    from deep_vision_amd.ops import bn as B

    torch.manual_seed(C + HW)
    N = 6
    xs = [torch.randn(N, C, HW, HW, device=DEV) * 2 + 0.5 for _ in range(3)]
    rs = [torch.randn(N, C, HW, HW, device=DEV) for _ in range(3)]
    dys = [torch.randn(N, C, HW, HW, device=DEV) for _ in range(3)]
    w0 = torch.empty(C, device=DEV).uniform_(0.5, 1.5)
    b0 = torch.empty(C, device=DEV).uniform_(-0.5, 0.5)

    def run(fuse):
        B.FUSE_FINALIZE = fuse
        try:
            bn = nn.BatchNorm2d(C).to(DEV)
            with torch.no_grad():
                bn.weight.copy_(w0)
                bn.bias.copy_(b0)
            outs = []
            n0, n1 = B.COUNTERS["bn_fin_fused"], B.COUNTERS["bn_bwd_fin_fused"]
            for x32, r32, dy in zip(xs, rs, dys):
                bn.weight.grad = bn.bias.grad = None
                x = _nhwc(x32).requires_grad_(True)
                r = _nhwc(r32).requires_grad_(True) if res else None
                y = F.batch_norm_act(x, bn, act, 0.1, residual=r, residual_post=res == "post")
                y.backward(_nhwc(dy))
                outs.append((y.detach().clone(), x.grad.clone(), bn.weight.grad.clone(), bn.bias.grad.clone(),
                             bn.running_mean.clone(), bn.running_var.clone()) + ((r.grad.clone(),) if res else ()))
            ws = bn.__dict__["_dv_ws"]
            shift = next(v for k, v in ws.items() if k[0] == "bn_fwd")[128].clone()
            return outs, shift, (B.COUNTERS["bn_fin_fused"] - n0, B.COUNTERS["bn_bwd_fin_fused"] - n1), bn
        finally:
            B.FUSE_FINALIZE = True

    fused, fshift, fcount, bn = run(True)
    plain, pshift, pcount, _ = run(False)
    assert fcount == (3, 3) and pcount == (0, 0)
    names = ("y", "dx", "dgamma", "dbeta", "running_mean", "running_var", "dres")
    for step, (a, b) in enumerate(zip(fused, plain)):
        for name, u, v in zip(names, a, b):
            assert torch.equal(u, v), (step, name, (u.float() - v.float()).abs().max().item())
    assert torch.equal(fshift, pshift)
    # the self-cleaning accumulators are zero again (shards) and the tickets are back to 0
    ws = bn.__dict__["_dv_ws"]
    for k, v in ws.items():
        if k[0] == "bn_fwd":
            assert not v[:128].any()
        elif k[0] in ("bn_bwd", "bn_fin_ticket"):
            assert not v.any()
    # fp32 torch reference of the last step
    ref = torch.nn.BatchNorm2d(C).to(DEV)
    with torch.no_grad():
        ref.weight.copy_(bn.weight)
        ref.bias.copy_(bn.bias)
    xr = _nhwc(xs[-1]).float().requires_grad_(True)
    z = ref(xr)
    if res and res != "post":
        z = z + _nhwc(rs[-1]).float()
    z = TF.relu(z) if act == "relu" else (TF.leaky_relu(z, 0.1) if act else z)
    if res == "post":
        z = z + _nhwc(rs[-1]).float()
    z.backward(_nhwc(dys[-1]).float())
    y, dx, dg, db = fused[-1][:4]
    rel = lambda a, b: ((a.float() - b.float()).norm() / b.float().norm()).item()  # noqa: E731
    assert rel(y, z) < 1e-2
    assert rel(dx, xr.grad) < 3e-2
    assert rel(dg, ref.weight.grad) < 1e-2
    assert rel(db, ref.bias.grad) < 1e-2
