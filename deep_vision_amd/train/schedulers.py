"""Learning-rate schedules of the reference.

* ``plateau`` / ``step`` / ``lambda``: torch.optim.lr_scheduler (the PT trainers step Plateau on
  validation top-1, mode 'max', R/ResNet/pytorch/train.py:411-415; Keras ReduceLROnPlateau on
  val_loss with patience 10 / min_lr 1e-5, R/ResNet/tensorflow/train.py:271-272).
* ``ManualPlateau``: the hand-rolled plateau of the TF2 loops (R/YOLO/tensorflow/train.py:56-68,
  R/Hourglass/tensorflow/train.py:46-58), reproduced counter for counter.
* ``LinearDecay``: constant, then linear to zero (R/CycleGAN/tensorflow/utils.py:5-28), stepped
  per optimizer step.
All of them act on ``optimizer.param_groups[*]['lr']`` and have state_dict / load_state_dict.
"""
from __future__ import annotations

import math

import torch

from ..config import LR_LAMBDAS


class ManualPlateau:
    """lr /= 10 once the patience counter exceeds ``max_patience``; the counter resets whenever
    the last validation loss is the lowest one. Call ``update(val_loss)`` after validation and
    ``step()`` at the start of every epoch (the reference's ``lr_decay()``)."""

    def __init__(self, optimizer, factor=0.1, max_patience=10, inclusive=False):
        self.optimizer = optimizer
        self.factor = factor
        self.max_patience = max_patience
        self.inclusive = inclusive  # Hourglass decays at >= max_patience, YOLO / CenterNet at >
        self.current_learning_rate = optimizer.param_groups[0]["lr"]
        self.last_val_loss = math.inf
        self.lowest_val_loss = math.inf
        self.patience_count = 0

    def update(self, val_loss: float) -> bool:
        """Record a validation loss; returns True when it is a new best."""
        self.last_val_loss = float(val_loss)
        best = self.last_val_loss < self.lowest_val_loss
        if best:
            self.lowest_val_loss = self.last_val_loss
        return best

    def step(self):
        if self.patience_count > self.max_patience or (self.inclusive and self.patience_count == self.max_patience):
            self.current_learning_rate *= self.factor
            self.patience_count = 0
        elif self.last_val_loss == self.lowest_val_loss:
            self.patience_count = 0
        self.patience_count += 1
        for g in self.optimizer.param_groups:
            g["lr"] = self.current_learning_rate

    def state_dict(self):
        return {k: v for k, v in self.__dict__.items() if k != "optimizer"}

    def load_state_dict(self, sd):
        self.__dict__.update(sd)


class LinearDecay:
    """lr(step) = lr0 for step < step_decay, else lr0 * (1 - (step - step_decay) / (total - step_decay))."""

    def __init__(self, optimizer, initial_learning_rate, total_steps, step_decay):
        self.optimizer = optimizer
        self.initial_learning_rate = initial_learning_rate
        self.total_steps = total_steps
        self.step_decay = step_decay
        self.step_count = 0
        self.current_learning_rate = initial_learning_rate
        self._apply()

    def lr_at(self, step: int) -> float:
        if step >= self.step_decay:
            return self.initial_learning_rate * (1 - 1 / (self.total_steps - self.step_decay) * (step - self.step_decay))
        return self.initial_learning_rate

    def _apply(self):
        self.current_learning_rate = self.lr_at(self.step_count)
        for g in self.optimizer.param_groups:
            g["lr"] = self.current_learning_rate

    def step(self):
        self.step_count += 1
        self._apply()

    def state_dict(self):
        return {k: v for k, v in self.__dict__.items() if k != "optimizer"}

    def load_state_dict(self, sd):
        self.__dict__.update(sd)
        self._apply()


def make_scheduler(name, optimizer, params, **ctx):
    """Build the scheduler of a config entry. ``ctx`` supplies ``steps_per_epoch`` / ``total_epochs``
    for LinearDecay."""
    params = dict(params or {})
    if name is None:
        return None
    if name == "plateau":
        params.pop("metric", None)
        return torch.optim.lr_scheduler.ReduceLROnPlateau(optimizer, **params)
    if name == "step":
        return torch.optim.lr_scheduler.StepLR(optimizer, **params)
    if name == "lambda":
        fn = params["lr_lambda"]
        return torch.optim.lr_scheduler.LambdaLR(optimizer, LR_LAMBDAS[fn] if isinstance(fn, str) else fn)
    if name == "manual_plateau":
        return ManualPlateau(optimizer, **params)
    if name == "linear_decay":
        spe = ctx["steps_per_epoch"]
        return LinearDecay(optimizer, optimizer.param_groups[0]["lr"], ctx["total_epochs"] * spe,
                           params.get("decay_epoch", 100) * spe)
    raise ValueError(f"unknown scheduler {name!r}")


def plateau_metric(params) -> str:
    return (params or {}).get("metric", "val_top1_acc")
