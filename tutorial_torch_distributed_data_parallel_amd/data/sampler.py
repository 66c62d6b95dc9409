"""Data sharding with the exact index semantics of the reference's samplers.

* :class:`DistributedSampler` -- torch's DistributedSampler (TORCH/utils/data/distributed.py:66-157,
  SURVEY.md §2.2 B9) as the reference uses it (REF/multi-GPU-training-torch.py:80-83,175-178):
  ``num_samples = ceil(N / world)`` (or floor with drop_last), shuffle with a generator seeded by
  ``seed + epoch`` (randperm), pad by wrapping to ``num_samples * world``, rank r takes
  ``indices[r::world]``; ``set_epoch`` only stores the epoch (without it the order repeats --
  the pitfall in REF/README.md:82-84). Bit-identical index lists to torch's sampler.
* :class:`BatchShardSampler` -- Accelerate's BatchSamplerShard with split_batches=False,
  even_batches=True (ACC/data_loader.py:110-272, B18): rank r takes every world-th *batch*; the
  tail loops back to the start so every rank yields the same number of batches.
"""
from __future__ import annotations

import math

import torch


class DistributedSampler(torch.utils.data.Sampler):
    def __init__(self, dataset, num_replicas: int | None = None, rank: int | None = None,
                 shuffle: bool = True, seed: int = 0, drop_last: bool = False):
        if num_replicas is None or rank is None:
            from ..parallel import runtime as rt

            num_replicas = rt.get_world_size() if num_replicas is None else num_replicas
            rank = rt.get_rank() if rank is None else rank
        if rank >= num_replicas or rank < 0:
            raise ValueError(f"Invalid rank {rank}, rank should be in [0, {num_replicas - 1}]")
        self.dataset = dataset
        self.num_replicas = num_replicas
        self.rank = rank
        self.epoch = 0
        self.drop_last = drop_last
        n = len(dataset)
        if drop_last and n % num_replicas != 0:
            self.num_samples = math.ceil((n - num_replicas) / num_replicas)
        else:
            self.num_samples = math.ceil(n / num_replicas)
        self.total_size = self.num_samples * num_replicas
        self.shuffle = shuffle
        self.seed = seed

    def indices(self) -> list:
        n = len(self.dataset)
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(n, generator=g).tolist()
        else:
            idx = list(range(n))
        if not self.drop_last:
            pad = self.total_size - len(idx)
            if pad <= len(idx):
                idx += idx[:pad]
            else:
                idx += (idx * math.ceil(pad / len(idx)))[:pad]
        else:
            idx = idx[: self.total_size]
        assert len(idx) == self.total_size
        idx = idx[self.rank: self.total_size: self.num_replicas]
        assert len(idx) == self.num_samples
        return idx

    def __iter__(self):
        return iter(self.indices())

    def __len__(self) -> int:
        return self.num_samples

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch


class BatchShardSampler(torch.utils.data.Sampler):
    """Whole batches of a base index order dealt round-robin to ranks (Accelerate semantics).

    Rank r yields batch i when i % world == r, but only once the whole round of `world` batches
    is complete. With even_batches the final partial round is completed by cycling through the
    first indices again, so every rank yields the same number of full batches.
    """

    def __init__(self, num_items: int, batch_size: int, num_replicas: int, rank: int,
                 drop_last: bool = False, even_batches: bool = True, order=None):
        self.n, self.bs = num_items, batch_size
        self.world, self.rank = num_replicas, rank
        self.drop_last, self.even = drop_last, even_batches
        self.order = order

    def _base_batches(self):
        idx = list(self.order) if self.order is not None else list(range(self.n))
        out = [idx[i: i + self.bs] for i in range(0, len(idx), self.bs)]
        if self.drop_last and out and len(out[-1]) < self.bs:
            out.pop()
        return out

    def __iter__(self):
        batches = self._base_batches()
        W, r, bs = self.world, self.rank, self.bs
        head = [i for b in batches[:W] for i in b] if not self.drop_last else []
        pending = None
        last_i, last = -1, []
        for i, b in enumerate(batches):
            if i % W == r:
                pending = b
            if i % W == W - 1 and len(b) == bs:
                yield pending
                pending = None
            last_i, last = i, b
        if self.drop_last or not head:
            return
        if not self.even:
            if pending:
                yield pending
            return
        if pending is not None and len(pending) == bs:
            yield pending
        while len(head) < W * bs:
            head = head + head
        i, cur = last_i, list(last)
        if len(cur) == bs:
            cur, i = [], i + 1
        pos = 0
        while i % W != 0 or cur:
            take = bs - len(cur)
            cur = cur + head[pos: pos + take]
            if i % W == r:
                yield cur
            pos += take
            cur, i = [], i + 1

    def __len__(self):
        return sum(1 for _ in iter(self))
