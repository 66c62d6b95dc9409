"""Sampler parity: DistributedSampler vs torch's, BatchShardSampler vs Accelerate's
BatchSamplerShard (both libraries are installed here and serve as oracles)."""
import pytest
import torch
from torch.utils.data import BatchSampler, SequentialSampler
from torch.utils.data import DistributedSampler as TorchDS

from tutorial_torch_distributed_data_parallel_amd.data import (BatchShardSampler, DeviceLoader,
                                                               DistributedSampler,
                                                               SyntheticDataset)


class _N:
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


@pytest.mark.parametrize("n", [10, 50000, 7, 1, 101])
@pytest.mark.parametrize("ws", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("shuffle", [True, False])
@pytest.mark.parametrize("drop_last", [False, True])
def test_distributed_sampler_matches_torch(n, ws, shuffle, drop_last):
    if drop_last and n < ws:
        pytest.skip("degenerate")
    for rank in range(ws):
        ours = DistributedSampler(_N(n), num_replicas=ws, rank=rank, shuffle=shuffle, seed=3,
                                  drop_last=drop_last)
        ref = TorchDS(_N(n), num_replicas=ws, rank=rank, shuffle=shuffle, seed=3,
                      drop_last=drop_last)
        for epoch in (0, 1, 5):
            ours.set_epoch(epoch)
            ref.set_epoch(epoch)
            assert list(ours) == list(ref)
            assert len(ours) == len(ref)


def test_set_epoch_pitfall():
    """SURVEY §4.3 oracle 5: without set_epoch the order repeats; with it, it changes;
    wrap-padding duplicates indices across ranks."""
    s = DistributedSampler(_N(10), num_replicas=3, rank=0, shuffle=True)
    a, b = list(s), list(s)
    assert a == b
    s.set_epoch(1)
    assert list(s) != a
    allidx = []
    for r in range(3):
        allidx += list(DistributedSampler(_N(10), num_replicas=3, rank=r, shuffle=True))
    assert len(allidx) == 12 and len(set(allidx)) == 10


@pytest.mark.parametrize("n,bs,ws", [(10, 3, 2), (50, 8, 4), (7, 2, 3), (64, 16, 4), (5, 4, 8),
                                     (100, 10, 3)])
@pytest.mark.parametrize("drop_last", [False, True])
@pytest.mark.parametrize("even", [True, False])
def test_batch_shard_matches_accelerate(n, bs, ws, drop_last, even):
    acc = pytest.importorskip("accelerate.data_loader")
    base = BatchSampler(SequentialSampler(range(n)), bs, drop_last)
    for rank in range(ws):
        ref = acc.BatchSamplerShard(base, num_processes=ws, process_index=rank,
                                    split_batches=False, even_batches=even)
        ours = BatchShardSampler(n, bs, ws, rank, drop_last=drop_last, even_batches=even)
        assert list(ours) == list(ref), (rank, list(ours), list(ref))


def test_device_loader_follows_sampler():
    ds = SyntheticDataset(40, (5,), 4, seed=1)
    s = DistributedSampler(ds, num_replicas=2, rank=1, shuffle=True)
    s.set_epoch(3)
    ld = DeviceLoader(ds, 6, sampler=s)
    idx = list(s)
    got = torch.cat([x for x, _ in ld])
    assert torch.equal(got, ds.x[idx])
    assert len(ld) == 4
    ld2 = DeviceLoader(ds, 6, sampler=s, drop_last=True)
    assert len(ld2) == 3 and sum(1 for _ in ld2) == 3


def test_synthetic_labels_learnable():
    ds = SyntheticDataset(200, (8,), 3, seed=0)
    assert ds.y.min() >= 0 and ds.y.max() < 3
    ds2 = SyntheticDataset(200, (8,), 3, seed=0)
    assert torch.equal(ds.x, ds2.x) and torch.equal(ds.y, ds2.y)
