"""GAN trainers: DCGAN (E10, R/DCGAN/tensorflow/main.py) and CycleGAN (E11,
R/CycleGAN/tensorflow/train.py), with ``ImagePool`` and ``LinearDecay`` (utils.py).

DCGAN: the reference computes both losses from one forward and applies both updates with the
*pre-update* discriminator. Native backward kernels accumulate parameter gradients directly
into the flat gradient buffers, so the two objectives are separated explicitly: the generator
loss is back-propagated first (discriminator gradients from it are discarded), then the
discriminator loss on ``fake.detach()``; both optimizers step afterwards -- the same update.

CycleGAN: generator step (6 G + 2 D forwards, LSGAN + 10 x cycle L1 + 5 x identity L1), the
fakes go through the 50-image history pools, then the discriminator step ((real + fake) / 2 per
discriminator); Adam(2e-4, beta1 .5) with per-step LinearDecay (constant for 100 epochs, then
linear to 0 at 200). The image pool keeps its history *on the device* (the reference round-trips
every image through the host eagerly).
Checkpoints: ``CheckpointManager`` (keep 3 / keep all) every 2 epochs with auto-restore.
"""
from __future__ import annotations

import argparse
import contextlib
import os
import random
import time

import numpy as np
import torch

from .. import models as M
from ..config import get_config
from ..data.loader import make_loader
from ..ops import loss as L
from ..utils.tensorboard import SummaryWriter
from . import checkpoint as C
from .engine import Engine, seed_everything
from .schedulers import LinearDecay


class ImagePool:
    """History buffer of generated images (R/CycleGAN/tensorflow/utils.py:32-61): until full,
    every image is stored and returned; afterwards with probability 1/2 a random stored image is
    returned (and replaced by the new one), else the new image itself."""

    def __init__(self, pool_size, rng: random.Random | None = None):
        self.pool_size = pool_size
        self.count = 0
        self.pool = []
        self.rng = rng or random.Random(0)

    def query(self, images):
        if self.pool_size == 0:
            return images
        out = []
        for image in images.detach():
            if self.count < self.pool_size:
                self.count += 1
                self.pool.append(image.clone())
                out.append(image)
            elif self.rng.uniform(0, 1) > 0.5:
                rid = self.rng.randint(0, self.pool_size - 1)
                tmp = self.pool[rid]
                self.pool[rid] = image.clone()
                out.append(tmp)
            else:
                out.append(image)
        y = torch.stack(out, 0)
        if images.dim() == 4 and images.stride(1) == 1:
            y = y.contiguous(memory_format=torch.channels_last)
        return y


def _no_sync(m):
    """Gradients of a network that must NOT be all-reduced in this backward (the discriminator
    during the generator step): the data-parallel hooks stay silent."""
    return m.no_sync() if hasattr(m, "no_sync") else contextlib.nullcontext()


# ------------------------------------------------------------------ DCGAN
class MnistImages(torch.utils.data.Dataset):
    """MNIST in [-1, 1] (28x28, main.py:21-26); synthetic digits when the IDX images are absent."""

    def __init__(self, root="../dataset", synthetic=False, n=1024):
        from ..data.datasets import read_idx, synthetic_digits

        p = os.path.join(root, "train-images-idx3-ubyte")
        if not synthetic and os.path.exists(p):
            imgs = read_idx(p)
        else:
            labels = np.random.default_rng(0).integers(0, 10, n)
            imgs = synthetic_digits(labels)
        self.x = torch.from_numpy((imgs.astype(np.float32) - 127.5) / 127.5).unsqueeze(1)

    def __len__(self):
        return len(self.x)

    def __getitem__(self, i):
        return self.x[i]


def train_dcgan(epochs=None, batch_size=None, data_dir="../dataset", synthetic=False, synthetic_size=1024,
                device=None, checkpoint_dir=None, max_steps=None, workers=0, seed=0):
    cfg = get_config("dcgan")
    eng = Engine(device=device)
    seed_everything(seed, eng.rank)
    bs = batch_size or cfg.batch_size
    noise_dim = cfg.extras["noise_dim"]
    ds = MnistImages(data_dir, synthetic, synthetic_size)
    loader = make_loader(ds, bs if eng.world == 1 else bs // eng.world, shuffle=True, num_workers=workers)
    G = eng.wrap(M.DCGANGenerator(noise_dim))
    D = eng.wrap(M.DCGANDiscriminator())
    opt_g = eng.optimizer("adam", G.parameters(), cfg.optimizer_params)
    opt_d = eng.optimizer("adam", D.parameters(), cfg.optimizer_params)
    mgr = C.CheckpointManager(checkpoint_dir or cfg.checkpoint_dir, max_to_keep=cfg.extras["keep"])
    step_var = 0
    for epoch in range(1, (epochs or cfg.total_epochs) + 1):
        start = time.time()
        G.train()
        D.train()
        for i, images in enumerate(loader):
            if max_steps is not None and i >= max_steps:
                break
            images = images.to(eng.device, non_blocking=True)
            noise = torch.randn(images.shape[0], noise_dim, device=eng.device)
            fake = G(noise)
            with _no_sync(D):
                g_loss = L.bce_with_logits(D(fake), 1.0)
                eng.backward_step(g_loss, G, opt_g)  # D gradients of g_loss are discarded below
            d_loss = L.bce_with_logits(D(images), 1.0) + L.bce_with_logits(D(fake.detach()), 0.0)
            eng.backward_step(d_loss, D, opt_d)
        step_var += 1
        if epoch % cfg.extras["save_every"] == 0:
            st = {"generator": C.strip_module_prefix(G.state_dict()), "discriminator": C.strip_module_prefix(D.state_dict()),
                  "generator_optimizer": opt_g.state_dict(), "discriminator_optimizer": opt_d.state_dict(),
                  "step": step_var, "rng": C.rng_state()}
            path = mgr.save(st)
            eng.log("Saved checkpoint for step {}: {}".format(step_var, path))
        eng.log("Time for epoch {} is {} sec".format(epoch, time.time() - start))
    eng.close()
    return mgr.latest_checkpoint


def dcgan_main(argv=None):
    ap = argparse.ArgumentParser(description="DCGAN on MNIST")
    ap.add_argument("--epochs", type=int, default=None)
    ap.add_argument("--batch-size", type=int, default=None)
    ap.add_argument("--data-dir", default="../dataset")
    ap.add_argument("--synthetic", action="store_true")
    ap.add_argument("--max-steps", type=int, default=None)
    ap.add_argument("--device", default=None)
    ap.add_argument("--checkpoint-dir", default=None)
    a = ap.parse_args(argv)
    return train_dcgan(a.epochs, a.batch_size, a.data_dir, a.synthetic, device=a.device,
                       checkpoint_dir=a.checkpoint_dir, max_steps=a.max_steps)


# ------------------------------------------------------------------ CycleGAN
class CycleGANDataset(torch.utils.data.Dataset):
    """Unpaired A/B streams (make_dataset, train.py:74-112): decode -> random flip -> resize 286 ->
    random crop 256 -> [-1, 1]. Pairs are drawn by index (zip of the two shuffled streams)."""

    def __init__(self, file_a, file_b, load=286, crop=256):
        from ..data.tfrecord import TFRecordIndex

        self.a, self.b = TFRecordIndex([file_a]), TFRecordIndex([file_b])
        self.load, self.crop = load, crop

    def __len__(self):
        return min(len(self.a), len(self.b))

    def _img(self, rec):
        from ..data.tfrecord import decode_example, example_values
        from ..data.yolo import decode_image, resize

        im = decode_image(example_values(decode_example(rec), "image/encoded")[0])
        if random.random() < 0.5:
            im = im[:, ::-1]
        im = resize(np.ascontiguousarray(im), (self.load, self.load))
        t, l = random.randint(0, self.load - self.crop), random.randint(0, self.load - self.crop)
        im = im[t:t + self.crop, l:l + self.crop].astype(np.float32) / 127.5 - 1
        return torch.from_numpy(np.ascontiguousarray(im.transpose(2, 0, 1)))

    def __getitem__(self, i):
        return self._img(self.a[i]), self._img(self.b[i])


class SyntheticPairs(torch.utils.data.Dataset):
    def __init__(self, n=8, size=256, seed=0):
        self.n, self.size, self.seed = n, size, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 7919 + i)
        return (torch.rand(3, self.size, self.size, generator=g) * 2 - 1,
                torch.rand(3, self.size, self.size, generator=g) * 2 - 1)


def train_cyclegan(dataset="horse2zebra", batch_size=4, epochs=None, synthetic=False, synthetic_size=8, size=256,
                   n_blocks=9, device=None, checkpoint_dir=None, max_steps=None, workers=0, tfrecord_dir="tfrecords",
                   seed=0, tensorboard_dir=None):
    cfg = get_config("cyclegan")
    ex = cfg.extras
    eng = Engine(device=device)
    seed_everything(seed, eng.rank)
    fa = os.path.join(tfrecord_dir, dataset, "trainA.tfrecord")
    fb = os.path.join(tfrecord_dir, dataset, "trainB.tfrecord")
    ds = SyntheticPairs(synthetic_size, size) if synthetic or not os.path.exists(fa) else CycleGANDataset(fa, fb)
    loader = make_loader(ds, int(batch_size), shuffle=True, num_workers=workers)
    total_batches = len(loader) if max_steps is None else min(len(loader), max_steps)
    eng.log("Batch size: {}, Total batches per epoch: {}".format(batch_size, total_batches))
    # each pair of networks shares one data-parallel wrapper (one flat gradient buffer per optimizer)
    gens = eng.wrap(torch.nn.ModuleList([M.CycleGANGenerator(n_blocks), M.CycleGANGenerator(n_blocks)]))
    diss = eng.wrap(torch.nn.ModuleList([M.CycleGANDiscriminator(), M.CycleGANDiscriminator()]))
    g_a2b, g_b2a = Engine.unwrap(gens)
    d_b, d_a = Engine.unwrap(diss)
    total_epochs = epochs or cfg.total_epochs
    opt_gen = eng.optimizer("adam", gens.parameters(), cfg.optimizer_params)
    opt_dis = eng.optimizer("adam", diss.parameters(), cfg.optimizer_params)
    decay = cfg.scheduler_params.get("decay_epoch", 100)
    gen_lr = LinearDecay(opt_gen, cfg.optimizer_params["lr"], total_epochs * total_batches, decay * total_batches)
    dis_lr = LinearDecay(opt_dis, cfg.optimizer_params["lr"], total_epochs * total_batches, decay * total_batches)
    mgr = C.CheckpointManager((checkpoint_dir or cfg.checkpoint_dir).format(dataset=dataset), max_to_keep=None)
    start_epoch = 1
    if mgr.latest_checkpoint:
        ck = C.load(mgr.latest_checkpoint)
        for m, k in ((g_a2b, "generator_a2b"), (g_b2a, "generator_b2a"), (d_b, "discriminator_b"), (d_a, "discriminator_a")):
            m.load_state_dict(ck[k])
        opt_gen.load_state_dict(ck["optimizer_gen"])
        opt_dis.load_state_dict(ck["optimizer_dis"])
        gen_lr.load_state_dict(ck["gen_lr"])
        dis_lr.load_state_dict(ck["dis_lr"])
        start_epoch = int(ck["epoch"]) + 1
        eng.log("Restored from {}".format(mgr.latest_checkpoint))
    else:
        eng.log("Initializing from scratch.")
    pool_b2a, pool_a2b = ImagePool(ex["pool_size"]), ImagePool(ex["pool_size"])
    lc, li = ex["lambda_cycle"], ex["lambda_identity"]
    # tf.keras.metrics.Mean x 10 + both learning rates -> TensorBoard once per epoch
    # (R/CycleGAN/tensorflow/train.py:267-312, logs/{dataset}/{ts}/train); the means accumulate on
    # the device (no per-step host sync)
    tb = SummaryWriter(os.path.join(tensorboard_dir or "logs", dataset, C.timestamp("%Y%m%d-%H%M%S"), "train"),
                       enabled=eng.is_main)
    metric_names = ("loss_gen_a2b", "loss_gen_b2a", "loss_dis_b", "loss_dis_a", "loss_id_a2b", "loss_id_b2a",
                    "loss_gen_total", "loss_dis_total", "loss_cycle_a2b2a", "loss_cycle_b2a2b")
    for epoch in range(start_epoch, total_epochs + 1):
        msum = torch.zeros(len(metric_names), dtype=torch.float64, device=eng.device)
        mcount = 0
        start = time.time()
        eng.log("Epoch {} starts. Learning rate: {}, {}".format(epoch, gen_lr.current_learning_rate,
                                                                dis_lr.current_learning_rate))
        gens.train()
        diss.train()
        for step, (real_a, real_b) in enumerate(loader):
            if max_steps is not None and step >= max_steps:
                break
            real_a = real_a.to(eng.device, non_blocking=True)
            real_b = real_b.to(eng.device, non_blocking=True)
            # ---- generators ----
            if hasattr(gens, "prepare"):
                gens.prepare()
            fake_a2b = g_a2b(real_a)
            recon_b2a = g_b2a(fake_a2b)
            fake_b2a = g_b2a(real_b)
            recon_a2b = g_a2b(fake_b2a)
            id_a2b = g_a2b(real_b)
            id_b2a = g_b2a(real_a)
            l_id_a2b, l_id_b2a = L.l1_loss(id_a2b, real_b), L.l1_loss(id_b2a, real_a)
            with _no_sync(diss):
                l_gen_a2b, l_gen_b2a = L.mse_loss(d_b(fake_a2b), 1.0), L.mse_loss(d_a(fake_b2a), 1.0)
                l_cyc_a, l_cyc_b = L.l1_loss(recon_b2a, real_a), L.l1_loss(recon_a2b, real_b)
                l_gen = l_gen_a2b + l_gen_b2a + (l_cyc_a + l_cyc_b) * lc + (l_id_a2b + l_id_b2a) * li
                eng.backward_step(l_gen, gens, opt_gen)
            gen_lr.step()
            # ---- discriminators on pooled fakes ----
            fb2a = pool_b2a.query(fake_b2a)
            fa2b = pool_a2b.query(fake_a2b)
            if hasattr(diss, "prepare"):
                diss.prepare()
            l_dis_a = (L.mse_loss(d_a(real_a), 1.0) + L.mse_loss(d_a(fb2a), 0.0)) * 0.5
            l_dis_b = (L.mse_loss(d_b(real_b), 1.0) + L.mse_loss(d_b(fa2b), 0.0)) * 0.5
            l_dis = l_dis_a + l_dis_b
            eng.backward_step(l_dis, diss, opt_dis)
            dis_lr.step()
            cur = dict(loss_gen_a2b=l_gen_a2b, loss_gen_b2a=l_gen_b2a, loss_dis_b=l_dis_b, loss_dis_a=l_dis_a,
                       loss_id_a2b=l_id_a2b, loss_id_b2a=l_id_b2a, loss_gen_total=l_gen, loss_dis_total=l_dis,
                       loss_cycle_a2b2a=l_cyc_a, loss_cycle_b2a2b=l_cyc_b)
            msum += torch.stack([cur[k].detach().double() for k in metric_names])
            mcount += 1
            if step % 10 == 0:
                vals = dict(loss_gen_a2b=l_gen_a2b, loss_gen_b2a=l_gen_b2a, loss_id_a2b=l_id_a2b, loss_id_b2a=l_id_b2a,
                            loss_cycle_a2b2a=l_cyc_a, loss_cycle_b2a2b=l_cyc_b, loss_gen_total=l_gen,
                            loss_dis_b=l_dis_b, loss_dis_a=l_dis_a, loss_dis_total=l_dis)
                eng.log("Epoch {} Step {} ".format(epoch, step),
                        " ".join("{}:{} ".format(k, float(v.detach())) for k, v in vals.items()))
        means = eng.reduce_sum((msum / max(1, mcount)).tolist())
        for k, v in zip(metric_names, means):
            tb.add_scalar(k, v / eng.world, epoch)
        tb.add_scalar("gen_learning_rate", gen_lr.current_learning_rate, epoch)
        tb.add_scalar("dis_learning_rate", dis_lr.current_learning_rate, epoch)
        if epoch % ex["save_every"] == 0:
            st = {"generator_a2b": C.strip_module_prefix(g_a2b.state_dict()),
                  "generator_b2a": C.strip_module_prefix(g_b2a.state_dict()),
                  "discriminator_b": C.strip_module_prefix(d_b.state_dict()),
                  "discriminator_a": C.strip_module_prefix(d_a.state_dict()),
                  "optimizer_gen": opt_gen.state_dict(), "optimizer_dis": opt_dis.state_dict(),
                  "gen_lr": gen_lr.state_dict(), "dis_lr": dis_lr.state_dict(), "epoch": epoch, "rng": C.rng_state()}
            path = mgr.save(st)
            eng.log("Saved checkpoint for epoch {}: {}".format(epoch, path))
        eng.log("Time for epoch {} is {} sec".format(epoch, time.time() - start))
    eng.log("Finished training.")
    tb.close()
    eng.close()
    return mgr.latest_checkpoint


def cyclegan_main(argv=None):
    ap = argparse.ArgumentParser(description="CycleGAN trainer")
    ap.add_argument("--dataset", help="The name of the dataset", required=True)
    ap.add_argument("--batch_size", "--batch-size", default="4", help="The batch size of input data")
    ap.add_argument("--epochs", type=int, default=None)
    ap.add_argument("--synthetic", action="store_true")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--max-steps", type=int, default=None)
    ap.add_argument("--device", default=None)
    ap.add_argument("--checkpoint-dir", default=None)
    ap.add_argument("--tfrecord-dir", default="tfrecords")
    ap.add_argument("--tensorboard-dir", default=None, help="TensorBoard root (default ./logs)")
    a = ap.parse_args(argv)
    return train_cyclegan(a.dataset, int(a.batch_size), a.epochs, a.synthetic, size=a.size, device=a.device,
                          checkpoint_dir=a.checkpoint_dir, max_steps=a.max_steps, tfrecord_dir=a.tfrecord_dir,
                          tensorboard_dir=a.tensorboard_dir)
