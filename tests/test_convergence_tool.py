"""tools/convergence.py streaming task: a batch is a pure function of (seed, step index), so the
native and reference arms of a long-horizon comparison see identical data (CPU)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def test_batches_are_deterministic_and_fresh():
    from convergence import Task

    t1 = Task(seed=3, classes=10, size=32, device="cpu")
    t2 = Task(seed=3, classes=10, size=32, device="cpu")
    x1, y1 = t1.batch(8, 5)
    x2, y2 = t2.batch(8, 5)
    assert torch.equal(x1, x2) and torch.equal(y1, y2)
    x3, _ = t1.batch(8, 6)
    assert not torch.equal(x1, x3)  # a new batch every step
    assert x1.shape == (8, 3, 32, 32) and y1.dtype == torch.int64
    assert set(y1.tolist()) <= set(t1.labels.tolist())


def test_templates_are_learnable_signal():
    """Images of one class correlate with their template far more than with another class's."""
    from convergence import Task

    t = Task(seed=0, classes=4, size=32, noise=1.0, shift=0, device="cpu")
    x, y = t.batch(64, 0)
    lab = {int(v): i for i, v in enumerate(t.labels.tolist())}
    own, other = [], []
    for img, lbl in zip(x, y.tolist()):
        c = lab[lbl]
        f = img.flatten()
        for k in range(4):
            tk = t.templ[k].flatten()
            corr = torch.dot(f, tk) / (f.norm() * tk.norm())
            (own if k == c else other).append(abs(corr.item()))
    assert sum(own) / len(own) > 3 * sum(other) / len(other)
