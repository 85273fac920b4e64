"""Device non-finite guard + checkpoint: the applied-step count (what Adam's bias
corrections follow) survives state_dict / load_state_dict when a step was skipped, instead of being
re-seeded from the host step count that also counts the skip."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_applied_step_count_survives_checkpoint_after_a_skip():
    from deep_vision_amd.train.optim import FusedAdam

    torch.manual_seed(0)
    p = torch.nn.Parameter(torch.randn(64, device=DEV))
    opt = FusedAdam([p], lr=1e-2)
    opt.use_device_guard(True)
    for g in (1.0, float("nan"), 1.0):  # the middle step is non-finite: skipped on the device
        opt.zero_grad()
        p.grad.fill_(g)
        opt.step()
    torch.cuda.synchronize()
    skipped, _, _ = opt.device_guard_counts()
    assert skipped == 1
    sd = opt.state_dict()
    assert sd["param_groups"][0]["_dv_applied"] == 2 and sd["param_groups"][0]["_dv_skipped"] == 1
    assert sd["param_groups"][0]["_dv_step"] == 3  # the host count includes the skip

    q = torch.nn.Parameter(p.detach().clone())
    opt2 = FusedAdam([q], lr=1e-2)
    opt2.load_state_dict(sd)
    opt2.use_device_guard(True)
    assert int(opt2._dguard[4].item()) == 2
    # guard created before the load: re-seeded from the saved applied count too
    opt3 = FusedAdam([torch.nn.Parameter(p.detach().clone())], lr=1e-2)
    opt3.use_device_guard(True)
    opt3.load_state_dict(sd)
    assert int(opt3._dguard[4].item()) == 2
