"""DataLoader wiring for one-process-per-GPU training.

* ``make_loader``: per-rank DataLoader; with a process group the dataset is sharded by a
  DistributedSampler (the reference's DataParallel split the *global* batch inside one process;
  here every rank loads its own ``global / world`` slice).
* ``make_loader(..., shm=True)``: the shared-memory batch ring (data/shm_loader.py) instead of
  the stock DataLoader -- workers write samples into pinned batch slots, nothing is pickled.
* ``DevicePrefetcher``: host->device copies of the next batch on a side HIP stream (pinned
  memory, non_blocking) while the current step computes; the consumer stream waits on an event
  and the tensors are ``record_stream``-ed so the caching allocator never recycles them early.
"""
from __future__ import annotations

import torch
from torch.utils.data import DataLoader
from torch.utils.data.distributed import DistributedSampler


def make_loader(dataset, batch_size, shuffle=True, num_workers=4, drop_last=False, seed=0, collate_fn=None,
                shm=False):
    import torch.distributed as dist

    if shm and num_workers > 0 and collate_fn is None:
        from .shm_loader import ShmBatchLoader

        return ShmBatchLoader(dataset, batch_size, num_workers=num_workers, shuffle=shuffle, drop_last=drop_last,
                              seed=seed)
    sampler = None
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        sampler = DistributedSampler(dataset, shuffle=shuffle, seed=seed, drop_last=drop_last)
        shuffle = False
    return DataLoader(dataset, batch_size=batch_size, shuffle=shuffle, sampler=sampler, num_workers=num_workers,
                      pin_memory=torch.cuda.is_available(), drop_last=drop_last, collate_fn=collate_fn,
                      persistent_workers=num_workers > 0)


def set_epoch(loader, epoch):
    if hasattr(loader, "set_epoch"):
        loader.set_epoch(epoch)
        return
    s = getattr(loader, "sampler", None)
    if isinstance(s, DistributedSampler):
        s.set_epoch(epoch)


def _to(obj, device, non_blocking):
    if torch.is_tensor(obj):
        return obj.to(device, non_blocking=non_blocking)
    if isinstance(obj, dict):
        return {k: _to(v, device, non_blocking) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to(v, device, non_blocking) for v in obj)
    return obj


def _record(obj, stream):
    if torch.is_tensor(obj) and obj.is_cuda:
        obj.record_stream(stream)
    elif isinstance(obj, dict):
        for v in obj.values():
            _record(v, stream)
    elif isinstance(obj, (list, tuple)):
        for v in obj:
            _record(v, stream)


class DevicePrefetcher:
    def __init__(self, loader, device):
        self.loader = loader
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(self.device) if self.cuda else None

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        it = iter(self.loader)
        nxt = self._load(it)
        while nxt is not None:
            batch, ev = nxt
            if ev is not None:
                cur = torch.cuda.current_stream(self.device)
                cur.wait_event(ev)
                _record(batch, cur)
            nxt = self._load(it)
            yield batch

    def _load(self, it):
        try:
            b = next(it)
        except StopIteration:
            return None
        if not self.cuda:
            return b, None
        owner, slot = getattr(b, "owner", None), getattr(b, "slot", -1)
        with torch.cuda.stream(self.stream):
            b = _to(b, self.device, True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        if owner is not None:  # a shared-memory ring slot: recycled once this copy has completed
            owner.copied(slot, ev)
        return b, ev
