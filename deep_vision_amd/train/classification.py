"""Supervised classification trainer (PT ImageNet / MNIST trainers E1-E3, TF1-Keras E4/E5, the
MobileNet TF2 skeleton E6 made runnable).

Same control flow and stdout protocol as R/ResNet/pytorch/train.py:310-538:
``validate(epoch 0)`` then per epoch ``train`` -> ``validate`` -> scheduler step (Plateau on
validation top-1, or on val_loss for the Keras configs) -> full checkpoint
``{name}-{ts}-epoch-{e}.pt``; every 10 batches
``Time, {ts}, Epoch: {e}, Batch: {b}, Training Loss: {avg10}, LR: {lr}``; after validation
``Epoch: {e}, Validation Top 1 acc: ...`` / ``Top 5 acc`` / ``Set Loss``.

MI355X-first differences: one process per GPU (global batch split across ranks, bucketed RCCL
all-reduce overlapped with backward), losses accumulate on the device and are read every 10
batches only, the 10-batch loss and validation sums are all-reduced in one packed
collective, Inception's auxiliary heads are trained with the GoogLeNet 0.3 weighting (A3).
"""
from __future__ import annotations

import argparse
import glob
import os
import pickle
import time

import torch

from .. import ops as F
from ..config import TrainConfig, get_config
from ..data import transforms as T
from ..data.datasets import ImageNet2012Dataset, MnistDataset, SyntheticClassification
from ..data.device_input import batch_images
from ..data.loader import DevicePrefetcher, make_loader, set_epoch
from ..utils.tensorboard import SummaryWriter
from . import checkpoint as C
from .engine import Engine, seed_everything
from .schedulers import make_scheduler, plateau_metric


def accuracy(output, target, topk=(1,)):
    """R/ResNet/pytorch/train.py:524-538 (pytorch/examples): percent correct in the top k."""
    with torch.no_grad():
        maxk = max(topk)
        batch = target.size(0)
        _, pred = output.float().topk(maxk, 1, True, True)
        pred = pred.t()
        correct = pred.eq(target.view(1, -1).expand_as(pred))
        return [correct[:k].reshape(-1).float().sum(0, keepdim=True).mul_(100.0 / batch) for k in topk]


def model_summary(model, input_shape) -> str:
    """A torchsummary-like header: parameter counts (trainable / total incl. BN statistics)."""
    n = sum(p.numel() for p in model.parameters())
    nt = sum(p.numel() for p in model.parameters() if p.requires_grad)
    nb = sum(b.numel() for k, b in model.named_buffers() if "running" in k)
    return (f"Model: {type(model).__name__}  input: {tuple(input_shape)}\n"
            f"Total params: {n + nb:,}\nTrainable params: {nt:,}\nNon-trainable params: {n + nb - nt:,}")


def _label_key(cfg):
    return "label" if cfg.dataset == "mnist" else "annotation"


def build_datasets(cfg: TrainConfig, data_dir=None, synthetic=False, synthetic_size=512, num_classes=None):
    key = _label_key(cfg)
    nc = num_classes or (10 if cfg.dataset == "mnist" else 1000)
    if cfg.dataset == "mnist":
        root = data_dir or "../dataset"
        mk = lambda split: MnistDataset(os.path.join(root, f"{split}-images-idx3-ubyte"),  # noqa: E731
                                        os.path.join(root, f"{split}-labels-idx1-ubyte"),
                                        synthetic_images=True,
                                        scale=255.0 if cfg.extras.get("scale_only") else 1.0,
                                        mean=(0.0,) if cfg.extras.get("scale_only") else (0.1307,),
                                        std=(1.0,) if cfg.extras.get("scale_only") else (0.3081,))
        if synthetic or not os.path.exists(os.path.join(root, "train-labels-idx1-ubyte")):
            return (SyntheticClassification(synthetic_size, cfg.input_shape, nc, key, seed=1),
                    SyntheticClassification(max(64, synthetic_size // 4), cfg.input_shape, nc, key, seed=2))
        return mk("train"), mk("t10k")
    if cfg.dataset == "imagenet" and not synthetic and cfg.extras.get("keras"):
        # TF1-Keras configs read the TFRecord shards (R/ResNet/tensorflow/train.py:226-235)
        root = data_dir or "../dataset"
        tr, va = os.path.join(root, "tfrecord", "tfrecord_train", "*"), os.path.join(root, "tfrecord", "tfrecord_val", "*")
        if glob.glob(tr) and glob.glob(va):
            from ..data.imagenet_tf import ImageNetTFRecordDataset

            return ImageNetTFRecordDataset(tr, True), ImageNetTFRecordDataset(va, False)
    if cfg.dataset == "imagenet" and not synthetic:
        root = data_dir or "../dataset"
        labels = os.path.join(root, "synsets.txt")
        tr, va = os.path.join(root, "train_flatten"), os.path.join(root, "val_flatten")
        if not os.path.isfile(labels):
            labels = None  # the packaged ImageNet-2012 synset list (data.imagenet_meta)
        if os.path.isdir(tr):
            dn = bool(cfg.extras.get("device_normalize", True))  # uint8 crops, normalised on the GPU
            # training crops: large JPEGs decoded at a reduced DCT scale (the pipeline rescales to 256
            # next anyway; a pre-filtered input to the cv2-geometry resize, a documented deviation
            # from the reference's full cv2.imread, README "Input pipeline"); validation keeps the
            # full decode so eval accuracy is measured on the reference's pixels
            ms = 256 if dn else None
            # ColorJitter draws in the worker, pixels jittered on the GPU (same bytes; README "Input pipeline")
            dj = dn and bool(cfg.extras.get("device_jitter", True))
            return (ImageNet2012Dataset(tr, labels, T.imagenet_train_transform(device_normalize=dn, device_jitter=dj),
                                        decode_min_side=ms),
                    ImageNet2012Dataset(va, labels, T.imagenet_val_transform(device_normalize=dn)))
    return (SyntheticClassification(synthetic_size, cfg.input_shape, nc, key, seed=1),
            SyntheticClassification(max(64, synthetic_size // 4), cfg.input_shape, nc, key, seed=2))


def _criterion(output, target, aux_weight):
    if isinstance(output, tuple):  # Inception V1 train mode: (main, aux1, aux2)
        main, *aux = output
        loss = F.cross_entropy(main, target)
        for a in aux:
            loss = loss + aux_weight * F.cross_entropy(a, target)
        return loss, main
    return F.cross_entropy(output, target), output


def train(loader, net, optimizer, epoch, loggers, eng: Engine, cfg: TrainConfig, max_steps=None, scheduler=None,
          epoch_stats=None):
    """``epoch_stats`` (Keras configs): a dict receiving the epoch's mean loss / top-1 / top-5 as
    fractions (the Keras History ``loss`` / ``acc`` / ``top_5_accuracy``)."""
    net.train()
    key = _label_key(cfg)
    aux_w = cfg.extras.get("aux_weight", 0.3)
    eng.log("Start training epoch {}".format(epoch))
    acc = torch.zeros((), device=eng.device)
    ep = torch.zeros(4, dtype=torch.float64, device=eng.device)  # loss sum, correct1, correct5, samples
    seen = 0
    for batch_i, data in enumerate(loader):
        if max_steps is not None and batch_i >= max_steps:
            break
        image = batch_images(data, eng.device)
        target = data[key].to(eng.device, dtype=torch.long, non_blocking=True)
        with eng.timer.step(samples=image.shape[0]):
            lr = C.get_lr(optimizer)
            loss, main = eng.train_step(net, optimizer, lambda im, t: _criterion(net(im), t, aux_w), image, target)
        if epoch_stats is not None:
            a1, a5 = accuracy(main.detach(), target, topk=(1, min(5, main.shape[1])))
            n = target.numel()
            ep += torch.stack([loss.detach().double() * n, a1[0].double() * n / 100, a5[0].double() * n / 100,
                               torch.tensor(float(n), dtype=torch.float64, device=eng.device)])
        acc += loss.detach().float()
        seen += 1
        if batch_i % 10 == 9:
            avg = eng.reduce_sum([acc.item() / 10.0])[0] / eng.world
            eng.log("Time, {}, Epoch: {}, Batch: {}, Training Loss: {}, LR: {}".format(
                C.timestamp(), epoch, batch_i + 1, avg, lr))
            C.log_metrics(loggers, "train_loss", avg, epoch)
            acc.zero_()
    if epoch_stats is not None:
        v = eng.reduce_sum(ep.tolist())
        n = max(1.0, v[3])
        epoch_stats.update(loss=v[0] / n, acc=v[1] / n, top_5_accuracy=v[2] / n)
    return seen


def keras_model_filename(cfg: TrainConfig, model_id: str) -> str:
    """``{name}-tf-{ts}`` (R/ResNet/tensorflow/train.py:258-260); the registry's ``_tf`` suffix is
    not part of the reference name."""
    name = cfg.name[:-3] if cfg.name.endswith("_tf") else cfg.name
    return "{}-tf-{}".format(name, model_id)


KERAS_LOGGER_KEYS = ("train_loss", "train_top1_acc", "train_top5_acc", "val_loss", "val_top1_acc", "val_top5_acc", "lr")


def keras_epoch_end(eng: Engine, model_dir: str, model_filename: str, loggers: dict, epoch: int, train_stats: dict,
                    val: tuple, lr: float, tb: SummaryWriter):
    """The reference's three Keras callbacks at ``on_epoch_end``: LoggersCallback (7 series, printed
    and pickled to ``{model_dir}{name}-tf-{ts}-loggers-epoch-{e}.pkl``, :81-144) and the
    TensorBoard callback's epoch scalars (:268-269, step = epoch index). Accuracies are fractions
    as in Keras; the checkpoint itself is written by the caller."""
    val_loss, top1, top5 = val
    vals = {"train_loss": train_stats.get("loss", float("nan")), "train_top1_acc": train_stats.get("acc", float("nan")),
            "train_top5_acc": train_stats.get("top_5_accuracy", float("nan")), "val_loss": val_loss,
            "val_top1_acc": top1 / 100.0, "val_top5_acc": top5 / 100.0, "lr": lr}
    for k in KERAS_LOGGER_KEYS:
        loggers.setdefault(k, {"epochs": [], "value": []})
        loggers[k]["epochs"].append(epoch)
        loggers[k]["value"].append(vals[k])
        eng.log("Epoch: {}, {}: {}".format(epoch, k, vals[k]))
    eng.log("Time: {}".format(C.timestamp()))
    for tag, k in (("loss", "train_loss"), ("acc", "train_top1_acc"), ("top_5_accuracy", "train_top5_acc"),
                   ("val_loss", "val_loss"), ("val_acc", "val_top1_acc"), ("val_top_5_accuracy", "val_top5_acc"),
                   ("lr", "lr")):
        tb.add_scalar(tag, vals[k], epoch - 1)
    if eng.is_main:
        os.makedirs(model_dir or ".", exist_ok=True)
        path = os.path.join(model_dir, "{}-loggers-epoch-{}.pkl".format(model_filename, epoch))
        tmp = path + ".tmp"
        with open(tmp, "wb") as f:
            pickle.dump({k: loggers[k] for k in KERAS_LOGGER_KEYS}, f, pickle.HIGHEST_PROTOCOL)
        os.replace(tmp, path)
        return path
    return None


def validate(loader, net, epoch, loggers, eng: Engine, cfg: TrainConfig, max_steps=None):
    net.eval()
    key = _label_key(cfg)
    tot = torch.zeros(6, dtype=torch.float64, device=eng.device)  # loss, top1, top5 (per-batch sums), n, c1, c5
    nbatches = 0
    with torch.no_grad():
        for batch_i, data in enumerate(loader):
            if max_steps is not None and batch_i >= max_steps:
                break
            image = batch_images(data, eng.device)
            target = data[key].to(eng.device, dtype=torch.long, non_blocking=True)
            out = net(image)
            out = out[0] if isinstance(out, tuple) else out
            loss = F.cross_entropy(out, target)
            a1, a5 = accuracy(out, target, topk=(1, min(5, out.shape[1])))
            n = target.numel()
            nbatches += 1
            tot += torch.stack([loss.double(), a1[0].double(), a5[0].double(), torch.tensor(float(n), device=eng.device,
                                dtype=torch.float64), a1[0].double() * n / 100, a5[0].double() * n / 100])
    vals = eng.reduce_sum(tot.tolist() + [nbatches])
    nb = max(1, vals[6])
    val_loss, top1, top5 = vals[0] / nb, vals[1] / nb, vals[2] / nb  # per-batch average
    eng.log("Epoch: {}, Validation Top 1 acc: {}".format(epoch, top1))
    eng.log("Epoch: {}, Validation Top 5 acc: {}".format(epoch, top5))
    eng.log("Epoch: {}, Validation Set Loss: {}".format(epoch, val_loss))
    if vals[3] > 0:
        eng.log("Epoch: {}, Validation exact Top 1 acc: {} ({} samples)".format(epoch, 100 * vals[4] / vals[3],
                                                                                  int(vals[3])))
    C.log_metrics(loggers, "val_top1_acc", top1, epoch)
    C.log_metrics(loggers, "val_top5_acc", top5, epoch)
    C.log_metrics(loggers, "val_loss", val_loss, epoch)
    return val_loss, top1, top5


def run_epochs(config: TrainConfig, checkpoint_path=None, *, device=None, data_dir=None, synthetic=False,
               epochs=None, max_steps=None, val_steps=None, synthetic_size=512, num_workers=None, seed=0,
               checkpoint_dir=None, profile=False, batch_size=None, tensorboard_dir=None, graph=False):
    eng = Engine(device=device, profile=profile, graph=graph)
    seed_everything(seed, eng.rank)
    eng.log("CUDA is available: {}".format(torch.cuda.is_available()))
    cfg = config
    if batch_size is not None:
        cfg = cfg.replace(batch_size=batch_size)
    bs = cfg.per_rank_batch(eng.world)
    train_ds, val_ds = build_datasets(cfg, data_dir, synthetic, synthetic_size)
    workers = cfg.num_workers if num_workers is None else num_workers
    # decoded-image sets go through the shared-memory batch ring (data/shm_loader.py: scales with
    # workers, no per-sample pickling); DV_SHM_LOADER=0 falls back to the stock DataLoader
    shm = isinstance(train_ds, ImageNet2012Dataset) and os.environ.get("DV_SHM_LOADER", "1") != "0"
    train_loader = make_loader(train_ds, bs, shuffle=True, num_workers=workers, seed=seed, shm=shm)
    val_loader = make_loader(val_ds, bs, shuffle=False, num_workers=workers, shm=shm)
    model = eng.build_model(cfg.model, **cfg.model_params)
    eng.log(model_summary(model, cfg.input_shape))
    net = eng.wrap(model)
    if eng.world > 1:
        eng.log("Using {} GPUs!".format(eng.world) if eng.device.type == "cuda" else f"Using {eng.world} ranks (gloo)")
    optimizer = eng.optimizer(cfg.optimizer, net.parameters(), cfg.optimizer_params)
    scheduler = make_scheduler(cfg.scheduler, optimizer, cfg.scheduler_params)
    loggers = C.initialize_loggers()
    model_dir = checkpoint_dir or cfg.checkpoint_dir
    model_id = time.strftime("%Y-%m-%dT%H:%M:%S", time.localtime())
    start_epoch = 1
    if checkpoint_path is not None:
        net, optimizer, scheduler, loggers, start_epoch = C.load_checkpoint(checkpoint_path, net, optimizer, scheduler,
                                                                            loggers)
    device_loader = DevicePrefetcher(train_loader, eng.device)
    keras = bool(cfg.extras.get("keras"))
    tb = None
    if keras:  # TF1-Keras configs: hdf5-style checkpoint names, pickled loggers, TensorBoard callback
        model_filename = keras_model_filename(cfg, model_id)
        kloggers = {}  # the LoggersCallback's own 7 series (pickled per epoch)
        tb = SummaryWriter(os.path.join(tensorboard_dir or "./tensorboard", model_filename), enabled=eng.is_main)
    else:
        validate(val_loader, net, 0, loggers, eng, cfg, val_steps)  # Keras fit() has no epoch-0 validation
    total = epochs if epochs is not None else cfg.total_epochs
    last = None
    for epoch in range(start_epoch, total + 1):
        set_epoch(train_loader, epoch)
        stats = {} if keras else None
        lr_epoch = C.get_lr(optimizer)
        train(device_loader, net, optimizer, epoch, loggers, eng, cfg, max_steps, epoch_stats=stats)
        val_loss, top1, top5 = validate(val_loader, net, epoch, loggers, eng, cfg, val_steps)
        if keras:
            keras_epoch_end(eng, model_dir, model_filename, kloggers, epoch, stats, (val_loss, top1, top5), lr_epoch, tb)
        if isinstance(scheduler, torch.optim.lr_scheduler.ReduceLROnPlateau):
            scheduler.step(val_loss if plateau_metric(cfg.scheduler_params) == "val_loss" else top1)
        elif scheduler is not None:
            scheduler.step()
        if keras:
            path = os.path.join(model_dir, "{}-checkpoint-epoch-{}.pt".format(model_filename, epoch))
        else:
            path = os.path.join(model_dir, C.classifier_checkpoint_name(cfg.name, model_id, epoch))
        last = C.atomic_save(C.training_state(epoch, net, optimizer, scheduler, loggers, config=cfg.name), path)
        if eng.timer.enabled:
            eng.log("[dv-profile] epoch {}: {}".format(epoch, eng.timer.summary()))
            eng.timer.reset()
    if tb is not None:
        tb.close()
    eng.barrier()
    eng.close()
    return last, loggers


def add_common_args(ap: argparse.ArgumentParser):
    ap.add_argument("-c", "--checkpoint", default=None, help="checkpoint to resume from ('latest' scans the dir)")
    ap.add_argument("--synthetic", action="store_true", help="synthetic data of the configured shape")
    ap.add_argument("--synthetic-size", type=int, default=512)
    ap.add_argument("--data-dir", default=None)
    ap.add_argument("--epochs", type=int, default=None, help="override total_epochs")
    ap.add_argument("--max-steps", type=int, default=None, help="batches per epoch (smoke runs)")
    ap.add_argument("--val-steps", type=int, default=None)
    ap.add_argument("--batch-size", type=int, default=None, help="override the configured batch")
    ap.add_argument("--workers", type=int, default=None)
    ap.add_argument("--device", default=None, help="cuda | cpu (default: cuda when available)")
    ap.add_argument("--checkpoint-dir", default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--profile", nargs="?", const="timer", default=None, choices=["timer", "rocprof"],
                    help="timer: per-phase HIP-event step timing; rocprof: re-run this command under "
                         "rocprofv3 --kernel-trace --stats (counters are collected in separate runs)")
    ap.add_argument("--tensorboard-dir", default=None, help="TensorBoard root (Keras configs: ./tensorboard)")
    ap.add_argument("--nproc", type=int, default=None,
                    help="spawn N ranks (one per GPU) via torch.distributed.run; default: every visible GPU "
                         "(the reference wraps the net in nn.DataParallel whenever > 1 GPU is visible)")
    ap.add_argument("--graph", action=argparse.BooleanOptionalAction, default=None,
                    help="capture the training step as a HIP graph and replay it (train/graph.py); default: "
                         "the model's measured-faster mode (deep_vision_amd/policy.py PREFERRED)")
    return ap


def resolve_checkpoint(arg, cfg, checkpoint_dir=None):
    if arg == "latest":
        if cfg.extras.get("keras"):
            base = cfg.name[:-3] if cfg.name.endswith("_tf") else cfg.name
            return C.latest(checkpoint_dir or cfg.checkpoint_dir, f"{base}-tf-*-checkpoint-epoch-*.pt")
        return C.latest(checkpoint_dir or cfg.checkpoint_dir, f"{cfg.name}-*.pt")
    return arg


def main(argv=None, choices=None, default=None):
    """``train.py -m <model> [-c <checkpoint>]`` (R/ResNet/pytorch/train.py:541-562)."""
    from ..launch import maybe_spawn

    ap = argparse.ArgumentParser(description="deep_vision_amd classification trainer")
    ap.add_argument("-m", "--model", choices=choices, default=default, required=default is None)
    add_common_args(ap)
    a = ap.parse_args(argv)
    if a.profile == "rocprof":
        from ..profiling import run_under_rocprof

        run_under_rocprof(argv)  # exits with the profiled child's status
    cfg = get_config(a.model)
    explicit = a.graph is not None
    a.graph = maybe_spawn(a.nproc, a.device, graph=a.graph, model=cfg.name)
    if a.graph and not explicit and (a.device == "cpu" or not torch.cuda.is_available()):
        a.graph = False  # the per-model default applies to the GPU path only
    ck = resolve_checkpoint(a.checkpoint, cfg, a.checkpoint_dir)
    run_epochs(cfg, ck, device=a.device, data_dir=a.data_dir, synthetic=a.synthetic, epochs=a.epochs,
               max_steps=a.max_steps, val_steps=a.val_steps, synthetic_size=a.synthetic_size, num_workers=a.workers,
               seed=a.seed, checkpoint_dir=a.checkpoint_dir, profile=a.profile == "timer", batch_size=a.batch_size,
               tensorboard_dir=a.tensorboard_dir, graph=a.graph)
