"""ops.common.fast_apply: the autograd Function entry without torch's per-call wrapper work gives
the same forward, gradients and saved-tensor behaviour as Function.apply (CPU)."""
import torch

from deep_vision_amd.ops.common import fast_apply


class _Cube(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, cfg):
        ctx.save_for_backward(x)
        ctx.k = k
        ctx.cfg = cfg
        return x * x * x * k

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return 3 * x * x * g * ctx.k, None, None


def test_fast_apply_matches_apply():
    x1 = torch.randn(5, dtype=torch.float64, requires_grad=True)
    x2 = x1.detach().clone().requires_grad_(True)
    y1 = _Cube.apply(x1, 2.0, ("a", 1))
    y2 = fast_apply(_Cube)(x2, 2.0, ("a", 1))
    assert torch.equal(y1, y2)
    y1.sum().backward()
    y2.sum().backward()
    assert torch.equal(x1.grad, x2.grad)
    assert y2.grad_fn is not None and type(y2.grad_fn).__name__.startswith("_Cube")


def test_fast_apply_gradcheck():
    x = torch.randn(4, dtype=torch.float64, requires_grad=True)
    f = fast_apply(_Cube)
    assert torch.autograd.gradcheck(lambda t: f(t, 1.5, None), (x,))
