"""Checkpoints, loggers and the reference's artefact naming.

One PyTorch-native mechanism for every family, always a full training state:
  PT classifiers  ``{checkpoint_dir}{name}-{%Y-%m-%dT%H:%M:%S}-epoch-{e}.pt`` with the reference
                  dict keys ``{epoch, model, optimizer, scheduler, loggers}`` (R/ResNet/pytorch/train.py:417-428)
  TF2 families    ``./models/model-v{version}-epoch-{e}-loss-{l:.4f}.pt`` (the ``.tf`` / ``.h5``
                  stems of R/YOLO/tensorflow/train.py:252-257, R/Hourglass/tensorflow/train.py:167-172);
                  the epoch is recovered from the name on resume (R/YOLO/tensorflow/train.py:302)
  GAN managers    ``{dir}/ckpt-{n}.pt`` with keep-N rotation (tf.train.CheckpointManager,
                  R/DCGAN/tensorflow/main.py:34-40, R/CycleGAN/tensorflow/train.py:133-148)
Extra keys (``rng``, ``world_size``, ``dtype``, ``framework``) are additive only. Writes happen
on rank 0 through a temp file + ``os.replace`` (atomic), loads accept ``module.``-prefixed state
dicts (DataParallel checkpoints) and the legacy ``loss_logger``/``acc_logger`` keys
(A18). Loading uses ``weights_only=True``: nothing in a checkpoint file is executed.
"""
from __future__ import annotations

import glob
import os
import re
import time
from typing import Dict, Optional

import torch

LOGGER_KEYS = ("train_loss", "val_loss", "val_top1_acc", "val_top5_acc")


def initialize_loggers(keys=LOGGER_KEYS) -> Dict[str, Dict[str, list]]:
    """R/ResNet/pytorch/train.py:260-279: {name: {'epochs': [], 'value': []}}."""
    return {k: {"epochs": [], "value": []} for k in keys}


def log_metrics(loggers, name, value, epoch):
    lg = loggers.setdefault(name, {"epochs": [], "value": []})
    lg["epochs"].append(epoch)
    lg["value"].append(float(value) if isinstance(value, (int, float)) or torch.is_tensor(value) else value)


def get_lr(optimizer) -> float:
    for g in optimizer.param_groups:
        return g["lr"]


def timestamp(fmt="%Y-%m-%dT%H:%M:%S") -> str:
    return time.strftime(fmt, time.localtime())


def classifier_checkpoint_name(name: str, model_id: str, epoch: int) -> str:
    return "{}-{}-epoch-{}.pt".format(name, model_id, epoch)


def best_model_name(version: str, epoch: int, loss: float) -> str:
    return "model-v{}-epoch-{}-loss-{:.4f}.pt".format(version, epoch, loss)


def epoch_from_name(path: str) -> int:
    """``model-v1.0.1-epoch-56-loss-42.0143.pt`` -> 56 (R/YOLO/tensorflow/train.py:302 uses
    ``int(path.split('-')[-3])``); also parses ``...-epoch-12.pt``."""
    m = re.search(r"epoch-(\d+)", os.path.basename(path))
    if not m:
        raise ValueError(f"no epoch in checkpoint name {path!r}")
    return int(m.group(1))


def strip_module_prefix(sd: dict) -> dict:
    if sd and all(k.startswith("module.") for k in sd):
        return {k[len("module."):]: v for k, v in sd.items()}
    return sd


def rng_state() -> dict:
    st = {"torch": torch.get_rng_state()}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        st["cuda"] = torch.cuda.get_rng_state()
    return st


def restore_rng(st: Optional[dict]) -> None:
    if not st:
        return
    if "torch" in st:
        torch.set_rng_state(st["torch"].cpu() if torch.is_tensor(st["torch"]) else st["torch"])
    if "cuda" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state(st["cuda"].cpu())


def _is_rank0() -> bool:
    import torch.distributed as dist

    return not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0


def atomic_save(obj, path: str) -> Optional[str]:
    """torch.save through ``path.tmp`` + os.replace, on rank 0 only. Returns the path (rank 0)."""
    if not _is_rank0():
        return None
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)
    return path


def training_state(epoch, model, optimizer=None, scheduler=None, loggers=None, **extra) -> dict:
    """Reference dict keys first, additive extras after."""
    import torch.distributed as dist

    st = {"epoch": epoch, "model": strip_module_prefix(model.state_dict())}
    st["optimizer"] = optimizer.state_dict() if optimizer is not None else None
    st["scheduler"] = scheduler.state_dict() if scheduler is not None else None
    st["loggers"] = loggers if loggers is not None else initialize_loggers()
    st["rng"] = rng_state()
    st["world_size"] = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    st["framework"] = "deep_vision_amd"
    st.update(extra)
    return st


def load(path: str, map_location="cpu") -> dict:
    ck = torch.load(path, map_location=map_location, weights_only=True)
    if "loggers" not in ck and ("loss_logger" in ck or "acc_logger" in ck):  # legacy GoogLeNet checkpoints
        ck["loggers"] = {"train_loss": ck.get("loss_logger"), "val_top1_acc": ck.get("acc_logger")}
    return ck


def load_checkpoint(path, net, optimizer=None, scheduler=None, loggers=None, strict=True):
    """R/ResNet/pytorch/train.py:293-307 semantics: restores model / optimizer / scheduler /
    loggers and returns ``start_epoch = epoch + 1``. Optimizer state follows the parameters'
    device (the reference moved it to CUDA by hand)."""
    ck = load(path)
    sd = ck["model"] if "model" in ck else ck
    net.load_state_dict(strip_module_prefix(sd), strict=strict)  # parallel.DataParallel forwards to .module
    if optimizer is not None and ck.get("optimizer") is not None:
        optimizer.load_state_dict(ck["optimizer"])
    if scheduler is not None and ck.get("scheduler") is not None:
        scheduler.load_state_dict(ck["scheduler"])
    if ck.get("loggers") is not None:
        loggers = ck["loggers"]
    restore_rng(ck.get("rng"))
    return net, optimizer, scheduler, loggers, int(ck.get("epoch", 0)) + 1


def latest(directory: str, pattern: str = "*.pt") -> Optional[str]:
    """Most recent checkpoint in ``directory`` (``--resume latest``): highest epoch in the name,
    else newest mtime."""
    files = [f for f in glob.glob(os.path.join(directory, pattern)) if not f.endswith(".tmp")]
    if not files:
        return None

    def key(f):
        try:
            return (epoch_from_name(f), os.path.getmtime(f))
        except ValueError:
            m = re.search(r"ckpt-(\d+)", f)
            return (int(m.group(1)) if m else -1, os.path.getmtime(f))

    return max(files, key=key)


class CheckpointManager:
    """tf.train.CheckpointManager equivalent: ``{dir}/ckpt-{n}.pt``, keep the newest ``max_to_keep``."""

    def __init__(self, directory: str, max_to_keep: Optional[int] = 3):
        self.directory = directory
        self.max_to_keep = max_to_keep

    def _existing(self):
        out = []
        for f in glob.glob(os.path.join(self.directory, "ckpt-*.pt")):
            m = re.search(r"ckpt-(\d+)\.pt$", f)
            if m:
                out.append((int(m.group(1)), f))
        return sorted(out)

    @property
    def latest_checkpoint(self) -> Optional[str]:
        ex = self._existing()
        return ex[-1][1] if ex else None

    def save(self, state: dict) -> Optional[str]:
        ex = self._existing()
        n = ex[-1][0] + 1 if ex else 1
        path = atomic_save(state, os.path.join(self.directory, f"ckpt-{n}.pt"))
        if path and self.max_to_keep:
            for _, f in self._existing()[:-self.max_to_keep]:
                os.remove(f)
        return path
