"""Custom-loop trainers of the TF2 families: YOLOv3 (E7), Stacked Hourglass (E8), CenterNet (E9).

Control flow of R/YOLO/tensorflow/train.py:122-257 / R/Hourglass/tensorflow/train.py:97-172:
per epoch ``lr_decay()`` (ManualPlateau), a training pass printing the reduced batch loss, a
validation pass (NaN batches skipped, as the Hourglass loop does), ``examples per second``,
weights saved as ``./models/model-v{version}-epoch-{e}-loss-{l:.4f}.pt`` on every new best
validation loss and at the end; ``--checkpoint`` resumes at ``epoch_from_name + 1``.

Loss scaling: the reference divides per-replica sums by the *global* batch
and SUM-all-reduces gradients. Here each rank divides by its *local* batch and the gradient
all-reduce averages (the 1/world is fused into the optimizer), which is the same update.
Reduced batch losses are read every ``log_every`` batches (the reference tf.prints every batch,
a device sync per step).

CenterNet's reference trainer has no loss; the paper's objective is used:
focal(heatmap) + 0.1 * L1(size) + L1(offset) at object centres, summed over stacks.
"""
from __future__ import annotations

import argparse
import glob
import math
import os
import time

import torch

from .. import ops as F
from ..config import TrainConfig, get_config
from ..data.loader import DevicePrefetcher, make_loader, set_epoch
from ..models.yolov3 import ANCHOR_MASKS, ANCHORS_WH
from ..ops import detection as Det
from ..ops import loss as L
from ..utils.tensorboard import SummaryWriter
from . import checkpoint as C
from .engine import Engine, seed_everything
from .schedulers import ManualPlateau


# ------------------------------------------------------------------ family losses
def yolo_loss(outputs, labels, num_classes):
    """Sum over the three scales of YoloLoss; returns (per-image summed total (scalar sum over the
    batch), components [xy, wh, class, obj] summed over the batch)."""
    comps = 0
    for out, y, m in zip(outputs, labels, ANCHOR_MASKS):
        comps = comps + Det.yolo_loss(out, y, ANCHORS_WH[list(m)], num_classes).sum(0)
    return comps.sum(), comps


def hourglass_loss(outputs, labels, fg_weight=81.0):
    """Sum over stacks of mean((y - y_hat)^2 (1 + 81 [y > 0])) (R/Hourglass/tensorflow/train.py:65-76)."""
    total = 0
    for o in outputs:
        total = total + L.heatmap_mse(o, labels, fg_weight)
    return total, None


def centernet_loss(outputs, labels, size_weight=0.1):
    hm, wh, off, mask = labels
    n = None
    total = 0
    for h, s, o in outputs:
        total = total + L.focal_loss(h, hm) + size_weight * L.masked_l1(s, wh, mask, n) + L.masked_l1(o, off, mask, n)
    return total, None


FAMILY_LOSS = {"yolo": "sum", "hourglass": "mean", "centernet": "mean"}


# ------------------------------------------------------------------ datasets
def _files(pattern):
    return sorted(glob.glob(pattern)) if pattern else []


def build_datasets(cfg: TrainConfig, train_glob=None, val_glob=None, synthetic=False, synthetic_size=64,
                   encode_on_device=False):
    """-> (train set, val set, collate). ``encode_on_device``: YOLO / Hourglass loaders ship raw
    ground truth and the targets are built on the GPU (ops.labels.device_targets)."""
    od = encode_on_device
    if cfg.family == "yolo":
        from functools import partial

        from ..data import yolo as Y

        nc = cfg.model_params.get("num_classes", 80)
        size = cfg.input_shape[1]
        tr, va = _files(train_glob), _files(val_glob)
        col = partial(Y.collate_raw, grids=tuple(size // s for s in (8, 16, 32))) if od else Y.collate
        if synthetic or not tr:
            return (Y.SyntheticYoloDataset(synthetic_size, nc, size, 1, encode_on_device=od),
                    Y.SyntheticYoloDataset(max(8, synthetic_size // 4), nc, size, 2, encode_on_device=od), col)
        return (Y.YoloTFRecordDataset(tr, True, nc, (size, size), encode_on_device=od),
                Y.YoloTFRecordDataset(va, False, nc, (size, size), encode_on_device=od), col)
    if cfg.family == "hourglass":
        from ..data import pose as P

        k = cfg.model_params.get("num_heatmap", 16)
        size = cfg.input_shape[1]
        hs = (size // 4, size // 4, k)
        tr, va = _files(train_glob), _files(val_glob)
        col = P.collate_raw if od else None
        if synthetic or not tr:
            return (P.SyntheticPoseDataset(synthetic_size, size, hs, 1, encode_on_device=od),
                    P.SyntheticPoseDataset(max(8, synthetic_size // 4), size, hs, 2, encode_on_device=od), col)
        return (P.MPIITFRecordDataset(tr, True, (size, size), hs, encode_on_device=od),
                P.MPIITFRecordDataset(va, False, (size, size), hs, encode_on_device=od), col)
    if cfg.family == "centernet":
        from ..data import centernet as CN

        nc = cfg.model_params.get("num_classes", 80)
        size = cfg.input_shape[1]
        return (CN.SyntheticCenterNetDataset(synthetic_size, nc, size, 1),
                CN.SyntheticCenterNetDataset(max(8, synthetic_size // 4), nc, size, 2), CN.collate)
    raise ValueError(cfg.family)


def _to_device(batch, device, cfg=None):
    imgs, labels = batch
    imgs = imgs.to(device, non_blocking=True)
    if isinstance(labels, dict):  # raw ground truth: targets built on the device
        from ..ops.labels import device_targets

        raw = {k: (v.to(device, non_blocking=True) if torch.is_tensor(v) else v) for k, v in labels.items()}
        k = cfg.model_params.get("num_heatmap", 16) if cfg is not None else 16
        hs = (imgs.shape[-1] // 4, imgs.shape[-2] // 4, k)
        nc = cfg.model_params.get("num_classes", 80) if cfg is not None else 80
        return imgs, device_targets(raw, nc, hs)
    if isinstance(labels, (tuple, list)):
        labels = tuple(t.to(device, non_blocking=True) for t in labels)
    else:
        labels = labels.to(device, non_blocking=True)
    return imgs, labels


class Trainer:
    def __init__(self, cfg: TrainConfig, eng: Engine, model, initial_epoch=1, epochs=None, log_every=10,
                 checkpoint_dir=None, tensorboard_dir=None):
        self.cfg = cfg
        self.eng = eng
        self.model = model
        self.initial_epoch = initial_epoch
        self.epochs = epochs or cfg.total_epochs
        self.log_every = log_every
        self.global_batch_size = cfg.global_batch(eng.world)
        self.optimizer = eng.optimizer(cfg.optimizer, model.parameters(), cfg.optimizer_params)
        self.plateau = ManualPlateau(self.optimizer, **cfg.scheduler_params)
        self.version = cfg.extras.get("version", "1.0.1")
        self.model_dir = checkpoint_dir or cfg.checkpoint_dir
        self.best_model = None
        self.nc = cfg.model_params.get("num_classes", 80)
        # TensorBoard streams with the reference's tags and directories (rank 0 only):
        # YOLO / CenterNet logs/gradient_tape/{ts}/{train,val} (R/YOLO/tensorflow/train.py:196-199),
        # Hourglass one writer in ./logs (R/Hourglass/tensorflow/train.py:134-157)
        ts = C.timestamp("%Y%m%d-%H%M%S")
        if cfg.family == "hourglass":
            self.tb_train = self.tb_val = SummaryWriter(tensorboard_dir or "./logs", enabled=eng.is_main)
        else:
            root = os.path.join(tensorboard_dir or "logs/gradient_tape", ts)
            self.tb_train = SummaryWriter(os.path.join(root, "train"), enabled=eng.is_main)
            self.tb_val = SummaryWriter(os.path.join(root, "val"), enabled=eng.is_main)
        self.total_steps = 0

    # ---- loss of one local batch, normalised for gradient averaging across ranks ----
    def compute_loss(self, outputs, labels, local_batch):
        fam = self.cfg.family
        if fam == "yolo":
            total, comps = yolo_loss(outputs, labels, self.nc)
            return total / local_batch, comps / local_batch
        if fam == "hourglass":
            total, _ = hourglass_loss(outputs, labels, self.cfg.extras.get("fg_weight", 81.0))
            return total / local_batch, None
        total, _ = centernet_loss(outputs, labels)
        return total, None

    def _forward_loss(self, images, labels):
        return self.compute_loss(self.model(images), labels, images.shape[0])

    def train_epoch(self, loader, epoch, max_steps=None):
        self.model.train()
        eng = self.eng
        acc = torch.zeros(5, device=eng.device)
        total = torch.zeros((), device=eng.device)
        nb = 0
        for i, batch in enumerate(loader):
            if max_steps is not None and i >= max_steps:
                break
            images, labels = _to_device(batch, eng.device, self.cfg)
            with eng.timer.step(samples=images.shape[0]):
                loss, comps = eng.train_step(self.model, self.optimizer, self._forward_loss, images, labels)
            nb += 1
            total += loss.detach().float()
            acc[0] += loss.detach().float()
            if comps is not None:
                acc[1:] += comps.detach().float()
            if nb % self.log_every == 0:
                v = eng.reduce_sum((acc / self.log_every).tolist())
                v = [x / eng.world for x in v]
                msg = "Trained batch: {} batch loss: {}".format(nb, v[0])
                step = self.total_steps + nb
                if self.cfg.family != "hourglass":
                    self.tb_train.add_scalar("batch train loss", v[0], step)
                if comps is not None:
                    msg += " batch xy loss {} batch wh loss {} batch obj loss {} batch_class_loss {}".format(
                        v[1], v[2], v[4], v[3])
                    for tag, val in (("batch xy loss", v[1]), ("batch wh loss", v[2]), ("batch obj loss", v[4]),
                                     ("batch class loss", v[3])):
                        self.tb_train.add_scalar(tag, val, step)
                eng.log(msg + " epoch total loss: {}".format(eng.reduce_sum([total.item()])[0] / eng.world))
                acc.zero_()
        return total, nb

    @torch.no_grad()
    def val_epoch(self, loader, max_steps=None):
        self.model.eval()
        eng = self.eng
        total, nb = 0.0, 0
        for i, batch in enumerate(loader):
            if max_steps is not None and i >= max_steps:
                break
            images, labels = _to_device(batch, eng.device, self.cfg)
            outputs = self.model(images)
            loss, _ = self.compute_loss(outputs, labels, images.shape[0])
            v = eng.reduce_sum([loss.item()])[0] / eng.world
            if math.isnan(v):  # R/Hourglass/tensorflow/train.py:126-130
                continue
            total += v
            nb += 1
        return total, nb

    def save_model(self, epoch, loss):
        path = os.path.join(self.model_dir, C.best_model_name(self.version, epoch, loss))
        st = C.training_state(epoch, self.model, self.optimizer, self.plateau, None, config=self.cfg.name)
        C.atomic_save(st, path)
        self.best_model = path
        self.eng.log("Model {} saved.".format(path))

    def run(self, train_loader, val_loader, max_steps=None, val_steps=None):
        eng = self.eng
        eng.log("{} Start training...".format(C.timestamp("%Y%m%d-%H%M%S")))
        for epoch in range(self.initial_epoch, self.epochs + 1):
            set_epoch(train_loader, epoch)
            t0 = time.time()
            self.plateau.step()
            eng.log("{} Started epoch {} with learning rate {}. Current LR patience count is {} epochs. "
                    "Last lowest val loss is {}.".format(C.timestamp("%Y%m%d-%H%M%S"), epoch,
                                                         self.plateau.current_learning_rate,
                                                         self.plateau.patience_count, self.plateau.lowest_val_loss))
            if self.cfg.family == "hourglass":
                self.tb_train.add_scalar("epoch learning rate", self.plateau.current_learning_rate, epoch)
            total, nb = self.train_epoch(DevicePrefetcher(train_loader, eng.device), epoch, max_steps)
            t1 = time.time()
            train_loss = eng.reduce_sum([total.item()])[0] / eng.world / max(nb, 1)
            self.total_steps += nb
            self.tb_train.add_scalar("epoch train loss", train_loss, epoch)
            eng.log("{} Epoch {} train loss {}, total train batches {}, {} examples per second".format(
                C.timestamp("%Y%m%d-%H%M%S"), epoch, train_loss, nb, nb * self.global_batch_size / (t1 - t0)))
            vt, vn = self.val_epoch(val_loader, val_steps)
            t2 = time.time()
            val_loss = vt / vn if vn else float("nan")
            self.tb_val.add_scalar("epoch val loss", val_loss, epoch)
            eng.log("{} Epoch {} val loss {}, total val batches {}, {} examples per second".format(
                C.timestamp("%Y%m%d-%H%M%S"), epoch, val_loss, vn, vn * self.global_batch_size / max(t2 - t1, 1e-9)))
            if self.plateau.update(val_loss):
                self.save_model(epoch, val_loss)
        self.save_model(self.epochs, self.plateau.last_val_loss)
        eng.log("{} Finished.".format(C.timestamp("%Y%m%d-%H%M%S")))
        self.tb_train.close()
        self.tb_val.close()
        return self.best_model


def train(cfg: TrainConfig, checkpoint=None, *, train_glob=None, val_glob=None, synthetic=False, synthetic_size=64,
          epochs=None, max_steps=None, val_steps=None, device=None, workers=2, log_every=10, checkpoint_dir=None,
          seed=None, batch_size=None, profile=False, tensorboard_dir=None, graph=False):
    eng = Engine(device=device, log_every=log_every, profile=profile, graph=graph)
    if eng.world > 1:  # MirroredStrategy's replica report (R/YOLO/tensorflow/train.py:282)
        eng.log(f"Using {eng.world} GPUs" if eng.device.type == "cuda" else f"Using {eng.world} ranks (gloo)")
    seed_everything(cfg.extras.get("seed", 0) if seed is None else seed, eng.rank)
    if batch_size:
        cfg = cfg.replace(batch_size=batch_size)
    from ..ops.common import backend

    on_dev = eng.device.type == "cuda" and backend() == "native" and cfg.extras.get("gpu_targets", True)
    tr, va, collate = build_datasets(cfg, train_glob, val_glob, synthetic, synthetic_size, encode_on_device=on_dev)
    bs = cfg.per_rank_batch(eng.world)
    train_loader = make_loader(tr, bs, shuffle=True, num_workers=workers, collate_fn=collate)
    val_loader = make_loader(va, bs, shuffle=False, num_workers=workers, collate_fn=collate)
    model = eng.build_model(cfg.model, **cfg.model_params)
    initial_epoch = 1
    if checkpoint:
        ck = C.load(checkpoint)
        model.load_state_dict(C.strip_module_prefix(ck["model"] if "model" in ck else ck))
        initial_epoch = C.epoch_from_name(checkpoint) + 1
        eng.log("Resume training from checkpoint {} and epoch {}".format(checkpoint, initial_epoch))
    net = eng.wrap(model)
    trainer = Trainer(cfg, eng, net, initial_epoch, epochs, log_every, checkpoint_dir, tensorboard_dir)
    best = trainer.run(train_loader, val_loader, max_steps, val_steps)
    eng.barrier()
    eng.close()
    return best


def add_args(ap):
    ap.add_argument("--synthetic", action="store_true")
    ap.add_argument("--synthetic-size", type=int, default=64)
    ap.add_argument("--epochs", type=int, default=None)
    ap.add_argument("--max-steps", type=int, default=None)
    ap.add_argument("--val-steps", type=int, default=None)
    ap.add_argument("--device", default=None)
    ap.add_argument("--workers", type=int, default=2)
    ap.add_argument("--log-every", type=int, default=10)
    ap.add_argument("--checkpoint-dir", default=None)
    ap.add_argument("--batch-size", type=int, default=None, help="per-replica batch")
    ap.add_argument("--input-size", type=int, default=None, help="square input size (default: the config's)")
    ap.add_argument("--profile", nargs="?", const="timer", default=None, choices=["timer", "rocprof"])
    ap.add_argument("--tensorboard-dir", default=None)
    ap.add_argument("--nproc", type=int, default=None,
                    help="processes (one per GPU); default: every visible GPU, like MirroredStrategy")
    ap.add_argument("--graph", action=argparse.BooleanOptionalAction, default=None,
                    help="HIP-graph replay of the whole training step, data-parallel all-reduces included "
                         "(default: the model's measured-faster mode, deep_vision_amd/policy.py -- on for YOLOv3 / "
                         "CenterNet / Hourglass; the captured step replays the eager one bit for bit in "
                         "deterministic mode, tests/test_branch_streams_gpu.py); --no-graph runs eagerly")
    return ap


def main(family_config: str, argv=None, tfrecords_default="./dataset/tfrecords"):
    """``train.py [--checkpoint PATH]`` (R/YOLO/tensorflow/train.py:276-313)."""
    from ..launch import maybe_spawn

    ap = argparse.ArgumentParser(description=f"deep_vision_amd {family_config} trainer")
    ap.add_argument("--checkpoint", type=str, help="checkpoint file path")
    ap.add_argument("--tfrecords", default=tfrecords_default, help="directory with train* / val* TFRecord shards")
    add_args(ap)
    a = ap.parse_args(argv)
    if a.profile == "rocprof":
        from ..profiling import run_under_rocprof

        run_under_rocprof(argv)
    a.graph = maybe_spawn(a.nproc, a.device, graph=a.graph, model=family_config)
    cfg = get_config(family_config)
    if a.input_size:
        cfg = cfg.replace(input_shape=(cfg.input_shape[0], a.input_size, a.input_size))
    return train(cfg, a.checkpoint, train_glob=os.path.join(a.tfrecords, "train*"),
                 val_glob=os.path.join(a.tfrecords, "val*"), synthetic=a.synthetic, synthetic_size=a.synthetic_size,
                 epochs=a.epochs, max_steps=a.max_steps, val_steps=a.val_steps, device=a.device, workers=a.workers,
                 log_every=a.log_every, checkpoint_dir=a.checkpoint_dir, batch_size=a.batch_size,
                 profile=a.profile == "timer", tensorboard_dir=a.tensorboard_dir, graph=a.graph)
