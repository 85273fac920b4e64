"""Shared-memory batch ring loader (data/shm_loader.py): every sample exactly once per epoch in
the sampler's order, the field schema, rank sharding, epoch re-seeding and worker-error reporting
(CPU: forked workers, no GPU)."""
import numpy as np
import pytest
import torch

from deep_vision_amd.data.shm_loader import ShmBatch, ShmBatchLoader


class _Toy(torch.utils.data.Dataset):
    def __init__(self, n=37, fail_at=None):
        self.n, self.fail_at = n, fail_at

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        if i == self.fail_at:
            raise ValueError(f"bad sample {i}")
        img = np.full((4, 5, 3), i % 251, dtype=np.uint8)
        return {"image": torch.from_numpy(img), "annotation": i, "flip": bool(i % 2),
                "jitter": float(np.random.random()), "name": f"s{i}"}


def _ids(batches):
    return [int(v) for b in batches for v in b["annotation"]]


@pytest.mark.parametrize("workers,bs", [(1, 8), (3, 8), (4, 5)])
def test_every_sample_once_in_sampler_order(workers, bs):
    ds = _Toy()
    ld = ShmBatchLoader(ds, bs, num_workers=workers, shuffle=True, seed=3, rank=0, world=1, pin=False)
    try:
        assert set(ld.schema) == {"image", "annotation", "flip", "jitter"}  # strings are not batched
        got = []
        for b in ld:
            assert isinstance(b, ShmBatch)
            n = len(b["annotation"])
            assert b["image"].shape == (n, 4, 5, 3) and b["image"].dtype == torch.uint8
            for k in range(n):  # the image of each row is its own sample's
                assert int(b["image"][k, 0, 0, 0]) == int(b["annotation"][k]) % 251
            assert b["flip"].dtype == torch.bool and b["jitter"].dtype == torch.float32
            got.append({k: v.clone() for k, v in b.items()})
        assert len(got) == len(ld) == -(-37 // bs)
        expect = torch.randperm(37, generator=torch.Generator().manual_seed(3)).tolist()
        assert _ids(got) == expect
    finally:
        ld.close()


def test_drop_last_and_second_epoch_reshuffles():
    ld = ShmBatchLoader(_Toy(), 8, num_workers=2, drop_last=True, seed=1, rank=0, world=1, pin=False)
    try:
        e0 = _ids([{k: v.clone() for k, v in b.items()} for b in ld])
        ld.set_epoch(1)
        e1 = _ids([{k: v.clone() for k, v in b.items()} for b in ld])
        assert len(e0) == len(e1) == 32 and e0 != e1
        assert sorted(e0) != list(range(32)) or e0 != e1
    finally:
        ld.close()


def test_rank_shards_partition_the_epoch():
    shards = []
    for r in range(3):
        ld = ShmBatchLoader(_Toy(), 4, num_workers=2, shuffle=True, seed=5, rank=r, world=3, pin=False)
        try:
            shards.append(_ids([{k: v.clone() for k, v in b.items()} for b in ld]))
        finally:
            ld.close()
    assert all(len(s) == 13 for s in shards)  # 37 padded to 39, 13 per rank
    assert set(shards[0]) | set(shards[1]) | set(shards[2]) == set(range(37))


def test_abandoned_iteration_then_full_epoch():
    ld = ShmBatchLoader(_Toy(), 4, num_workers=3, shuffle=False, rank=0, world=1, pin=False)
    try:
        for i, _ in enumerate(ld):
            if i == 1:
                break
        assert _ids([{k: v.clone() for k, v in b.items()} for b in ld]) == list(range(37))
    finally:
        ld.close()


def test_worker_error_is_raised_in_the_main_process():
    ld = ShmBatchLoader(_Toy(fail_at=9), 4, num_workers=2, shuffle=False, rank=0, world=1, pin=False)
    with pytest.raises(RuntimeError, match="bad sample 9"):
        for _ in ld:
            pass
    ld.close()


def test_make_loader_shm_and_prefetcher_on_cpu():
    from deep_vision_amd.data.loader import DevicePrefetcher, make_loader, set_epoch

    ld = make_loader(_Toy(), 8, shuffle=False, num_workers=2, shm=True)
    try:
        assert isinstance(ld, ShmBatchLoader)
        set_epoch(ld, 2)
        assert ld.epoch == 2
        got = [int(v) for b in DevicePrefetcher(ld, "cpu") for v in b["annotation"]]
        assert got == list(range(37))
    finally:
        ld.close()
