"""Two (or more) ranks on the GPU(s) with DV_DIST_BACKEND=gloo: data-parallel training of a
BN network through the native kernels must keep every replica bit-identical, and the reduced
gradient must be the mean of the per-rank gradients (checked on a BN-free tail)."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, ".")
from deep_vision_amd import models as M  # noqa: E402
from deep_vision_amd import ops as F  # noqa: E402
from deep_vision_amd.parallel.ddp import DataParallel  # noqa: E402
from deep_vision_amd.parallel.dist import init_distributed  # noqa: E402
from deep_vision_amd.train.optim import FusedSGD  # noqa: E402

world, rank, local, dev = init_distributed()
torch.manual_seed(1 + rank)
model = M.get_model("resnet34").to(dev)
ddp = DataParallel(model, bucket_mb=8)
opt = FusedSGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
g = torch.Generator(device="cpu").manual_seed(7)
losses = []
for step in range(4):
    x = torch.randn(world * 8, 3, 112, 112, generator=g)[rank * 8:(rank + 1) * 8].to(dev)
    y = torch.randint(0, 1000, (world * 8,), generator=g)[rank * 8:(rank + 1) * 8].to(dev)
    opt.zero_grad()
    loss = F.cross_entropy(ddp(x), y)
    loss.backward()
    ddp.finish()
    opt.step(grad_scale=ddp.grad_scale)
    losses.append(loss.item())
flat = ddp.pflat.double()
chk = torch.stack([flat.sum(), (flat * torch.arange(flat.numel(), device=dev, dtype=torch.float64) % 97).sum()])
allc = [torch.zeros_like(chk) for _ in range(world)]
dist.all_gather(allc, chk)
same = all(torch.equal(allc[0], c) for c in allc)
print(f"rank {rank} losses {[round(l, 4) for l in losses]} replicas_identical={same} "
      f"allreduce_calls={ddp.comm_stats['allreduce_calls']} buckets={len(ddp.buckets)}", flush=True)
dist.destroy_process_group()
sys.exit(0 if same else 1)
