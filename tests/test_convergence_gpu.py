"""Training-trajectory checks of the native step (SURVEY §7.3 phase 2), native HIP kernels vs
PyTorch under autocast bf16 from one initialisation, SGD momentum 0.9 / wd 1e-4.

The native arm runs in deterministic mode (``set_deterministic``): no float-atomic accumulation
order, so its trajectory is bitwise reproducible run to run and box to box, and a bound that holds
once holds always. Bounds are placed only where they are well-posed (profiles/agreement_r6.txt,
tools/agreement.py, 3 seeds per regime):
- per-step agreement with torch-bf16 over the first steps, before rounding differences are
  amplified (max relative loss difference measured: 1.7 % over 20 steps at lr .01 / noise .3,
  2.1 % over 10 steps at lr .02 / noise 1.0, 0.9 % over 20 steps for MobileNet) -- bounded at ~3x;
- final convergence only in the well-conditioned regime (lr .01-.02 / noise .3), where the torch arm
  itself clears the bound with a wide margin. The lr .02 / noise 1.0 and lr .1 streaming regimes are
  chaotic in BOTH arms (per-step differences of 27-66 % by step 20 between two correct bf16
  implementations), so there only agreement before the divergence and "it trains" are asserted.
Reference oracle: a completed run that trains (R/ResNet/pytorch/logs/resnet34-yanjiali-010319.log).
"""
import math
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def _rel(a, b):
    return [abs(x - y) / max(abs(y), 1e-3) for x, y in zip(a, b)]


@pytest.mark.parametrize("name,bs,lr", [("resnet50", 64, 0.01), ("mobilenet1", 64, 0.02)])
def test_learnable_task_converges(name, bs, lr):
    """Well-conditioned regime: both arms drive the cross-entropy from ln(1000) to ~0 in 100 steps,
    and the first 20 steps agree per step."""
    from loss_curve import run_curve

    curves = run_curve(name, bs=bs, steps=100, lr=lr, task="learnable", noise=0.3, deterministic=True)
    nat, ref = curves["native"], curves["torch-bf16"]
    assert all(math.isfinite(v) for v in nat)
    assert nat[0] > 5.0 and ref[0] > 5.0          # starts at ~ln(1000)
    d = _rel(nat[:20], ref[:20])
    assert max(d) < 0.05, [round(v, 4) for v in d]
    tail_n = sum(nat[-10:]) / 10
    tail_r = sum(ref[-10:]) / 10
    assert tail_r < 0.1, f"reference did not learn: {ref[::10]}"
    assert tail_n < 0.1, f"native did not learn: {nat[::10]}"


@pytest.mark.parametrize("seed", [0, 1])
def test_resnet50_high_noise_early_agreement(seed):
    """lr .02 / noise 1.0: the first 10 steps agree per step within 6 % (measured <= 2.1 %); after
    that both arms pass through loss spikes whose timing is set by rounding. The native arm is
    bitwise reproducible (two deterministic runs give the same 10 losses)."""
    from loss_curve import run_curve

    c = run_curve("resnet50", bs=64, steps=10, lr=0.02, task="learnable", noise=1.0, seed=seed, deterministic=True)
    c2 = run_curve("resnet50", bs=64, steps=10, lr=0.02, task="learnable", noise=1.0, seed=seed, deterministic=True,
                   arms=("native",))
    assert all(math.isfinite(v) for v in c["native"])
    assert c["native"] == c2["native"], (c["native"], c2["native"])
    d = _rel(c["native"], c["torch-bf16"])
    assert max(d) < 0.06, [round(v, 4) for v in d]


@pytest.mark.parametrize("seed", [0, 1])
def test_resnet50_streaming_task_trains(seed):
    """The reference SGD settings (lr .1, momentum .9, wd 1e-4) on the streaming learnable task (a
    fresh batch every step; profiles/convergence_resnet50.txt has the 1,000-step curves): the
    initial losses agree, and over 200 steps the native run leaves ln(1000) ~ 6.9 well behind (the
    trajectory itself is chaotic from step ~2 in both arms: 14-19 % apart at step 5)."""
    from convergence import run

    r = run("resnet50", bs=128, steps=200, lr=0.1, seed=seed, every=100, n_eval=256, log=lambda s: None,
            deterministic=True)
    nat, ref = r["native"], r["torch-bf16"]
    assert all(math.isfinite(v) for v in nat["loss"])
    assert abs(nat["loss"][0] - ref["loss"][0]) / ref["loss"][0] < 0.01, (nat["loss"][:3], ref["loss"][:3])
    ln, lr_ = nat["checkpoints"][-1]["train_loss"], ref["checkpoints"][-1]["train_loss"]
    assert lr_ < 6.0, f"reference did not train: {lr_}"
    assert ln < 5.5, (ln, lr_)
