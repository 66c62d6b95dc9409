"""Synthetic datasets resident in device memory, plus a device-side loader.

The reference trains on CIFAR-10 resized to 224x224 through torchvision, downloaded concurrently
by every rank (REF/data_and_toy_model.py:8-38; SURVEY.md §5.2 download race) and decoded by 2
worker processes per rank (REF/multi-GPU-training-torch.py:85-99). There is no network here and
the benchmark is defined on synthetic data, so a dataset is a tensor already in HBM (288 GB per
MI355X) and a batch is a gather by the sampler's indices: no host decode, no pinned H2D copy
per step. Labels are a fixed random linear function of the input so a
model can actually learn (loss curves are meaningful in tests).
"""
from __future__ import annotations


import torch


class SyntheticDataset(torch.utils.data.Dataset):
    """`n` samples of `shape` (float32) with labels in [0, num_classes), built from `seed`."""

    def __init__(self, n: int, shape, num_classes: int = 10, seed: int = 0, device="cpu",
                 learnable: bool = True, dtype=torch.float32):
        self.n = int(n)
        self.shape = tuple(shape)
        self.num_classes = num_classes
        device = torch.device(device)
        g = torch.Generator(device=device if device.type == "cuda" else "cpu")
        g.manual_seed(seed)
        self.x = torch.randn((self.n,) + self.shape, generator=g, device=device, dtype=dtype)
        if learnable:
            feat = self.x.reshape(self.n, -1)
            proj = torch.randn(feat.shape[1], num_classes, generator=g, device=device,
                               dtype=dtype)
            self.y = (feat @ proj).argmax(dim=1)
        else:
            self.y = torch.randint(0, num_classes, (self.n,), generator=g, device=device)
        self.device = device
        if device.type == "cuda" and dtype == torch.float32 and len(self.shape) == 3 and \
                self.shape[0] % 4 != 0:
            self.x = padded_channels_last(self.x)

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return self.x[i], self.y[i]


def padded_channels_last(x: torch.Tensor) -> torch.Tensor:
    """``x`` [n, C, H, W] (C % 4 != 0, e.g. RGB) re-laid out as channels_last with the channel
    stride rounded up to a multiple of 4 (zero-filled): a [n, C, H, W] view of a
    [n, H, W, Cp] buffer. The NHWC convolutions read it in place (16-B chunks of 4 channels per
    pixel, ops/conv.py) instead of re-packing every batch; values and shape are unchanged."""
    n, c, h, w = x.shape
    cp = (c + 3) // 4 * 4
    base = torch.zeros((n, h, w, cp), device=x.device, dtype=x.dtype)
    base[..., :c] = x.permute(0, 2, 3, 1)
    return _padded_view(base, c)


def _padded_view(base: torch.Tensor, c: int) -> torch.Tensor:
    n, h, w, cp = base.shape
    v = base.as_strided((n, c, h, w), (h * w * cp, 1, w * cp, cp))
    v._tdp_padded_base = base  # the zero-filled [n, H, W, Cp] storage (ops/conv.py reads it)
    return v


def gather_batch(x: torch.Tensor, y: torch.Tensor, idx: torch.Tensor):
    """``(x[idx], y[idx])``: on the GPU one native launch for samples and labels
    (csrc/elementwise.hip ``gather_batch``), else two ``index_select``. A channel-padded
    channels_last dataset (``padded_channels_last``) yields a batch in the same layout."""
    base = getattr(x, "_tdp_padded_base", None)
    if base is not None and x.is_cuda and idx.is_cuda and len(idx) > 0:
        from .._native import native

        xb, yb = native().gather_batch(base, y, idx)
        return _padded_view(xb, x.shape[1]), yb
    if (x.is_cuda and idx.is_cuda and x.dtype == torch.float32 and y.dtype == torch.long and
            idx.dtype == torch.long and x.is_contiguous() and y.is_contiguous() and
            idx.is_contiguous() and y.device == x.device and len(idx) > 0):
        from .._native import native
        from ..ops.linear import attach_planes, planes_input_fit

        if x.dim() == 2 and planes_input_fit(len(idx), x.shape[1]):
            # a feature batch for a skinny Linear: its bf16 split planes come out of the same
            # launch (ops/linear.py planes GEMM)
            r = native().gather_batch(x, y, idx, planes=True)
            if len(r) == 3:
                attach_planes(r[0], r[2])
            return r[0], r[1]
        xb, yb = native().gather_batch(x, y, idx)
        return xb, yb
    return x.index_select(0, idx), y.index_select(0, idx)


class EpochCursor:
    """Device-side batch position over one epoch's sample order, for captured steps.

    The planes gather (csrc/gemm_planes.hip ``gather_planes_kernel``, cursor form) reads its
    batch from ``order[pos : pos + batch]`` and advances ``pos`` itself (the last workgroup to
    finish), so every replay of a captured step gathers the next batch without a per-step index
    copy. The host installs each epoch's order with ``set_order`` (one copy per epoch, stream
    ordered before the next replay), which also rewinds the position."""

    def __init__(self, capacity: int, batch: int, device):
        self.order = torch.zeros(capacity, dtype=torch.long, device=device)
        # {position, arrivals, per-row slice arrivals [batch]} (all re-armed by the kernel); the
        # per-row counters let several workgroups share a row
        rows = int(batch)
        self.state = torch.zeros(2 + rows, dtype=torch.long, device=device)
        self.batch = int(batch)

    def set_order(self, idx: torch.Tensor) -> None:
        n = len(idx)
        if n > len(self.order):
            raise ValueError(f"epoch order of {n} exceeds the cursor capacity {len(self.order)}")
        self.order[:n].copy_(idx)
        if n < len(self.order):
            self.order[n:].fill_(int(idx[-1]) if idx.device.type == "cpu" else 0)
        self.state.zero_()

    @staticmethod
    def fits(x: torch.Tensor, y: torch.Tensor, batch: int) -> bool:
        """The dataset can use the cursor gather (a 2-D fp32 feature table for a skinny Linear)."""
        from ..ops.linear import planes_input_fit

        return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and x.is_contiguous() and
                y.dtype == torch.long and y.is_contiguous() and x.shape[1] % 4 == 0 and
                planes_input_fit(batch, x.shape[1]))


def gather_batch_cursor(x: torch.Tensor, y: torch.Tensor, cur: EpochCursor):
    """``gather_batch`` of the cursor's next batch (advances the device-side position)."""
    from .._native import native
    from ..ops.linear import attach_planes

    xb, yb, p = native().gather_batch(x, y, cur.order, planes=True, cursor=cur.state,
                                      batch=cur.batch)
    attach_planes(xb, p)
    return xb, yb


class DeviceLoader:
    """Iterates (inputs, labels) batches of a tensor dataset by sampler order, on device.

    ``sampler`` is any iterable of indices (e.g. DistributedSampler) and is re-iterated every
    epoch, so ``sampler.set_epoch(e)`` takes effect exactly as with torch's DataLoader. The index
    list of an epoch goes to the device once; each batch is one ``index_select`` per tensor.
    """

    def __init__(self, dataset, batch_size: int, sampler=None, drop_last: bool = False,
                 device=None, batch_sampler=None):
        self.dataset = dataset
        self.batch_size = batch_size
        self.sampler = sampler
        self.batch_sampler = batch_sampler
        self.drop_last = drop_last
        self.device = torch.device(device) if device is not None else dataset.device

    def epoch_indices(self) -> torch.Tensor:
        """The whole epoch's index order as ONE device tensor (one host->device copy per epoch,
        never a pageable copy per step, which would serialise the CPU with the GPU queue)."""
        if self.batch_sampler is not None:
            flat = [i for b in self.batch_sampler for i in b]
        else:
            flat = list(self.sampler) if self.sampler is not None else \
                list(range(len(self.dataset)))
        idx = torch.as_tensor(flat, dtype=torch.long)
        dev = self.dataset.x.device
        if dev.type == "cuda":
            idx = idx.pin_memory().to(dev, non_blocking=True)
        return idx

    def _index_batches(self):
        idx = self.epoch_indices()
        if self.batch_sampler is not None:
            s = 0
            for b in self.batch_sampler:
                yield idx[s: s + len(b)]
                s += len(b)
            return
        n = len(idx)
        stop = n - (n % self.batch_size) if self.drop_last else n
        for s in range(0, stop, self.batch_size):
            yield idx[s: s + self.batch_size]

    def __iter__(self):
        x, y = self.dataset.x, self.dataset.y
        for b in self._index_batches():
            xb, yb = gather_batch(x, y, b)
            if xb.device != self.device:
                xb = xb.to(self.device, non_blocking=True)
                yb = yb.to(self.device, non_blocking=True)
            yield xb, yb

    def __len__(self):
        if self.batch_sampler is not None:
            return len(self.batch_sampler)
        n = len(self.sampler) if self.sampler is not None else len(self.dataset)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)


def cifar_like(n_train: int = 50000, n_test: int = 10000, shape=(3, 224, 224), device="cpu",
               seed: int = 0):
    """Train/test sets with the reference's tensor shapes (CIFAR-10 resized to 224)."""
    return (SyntheticDataset(n_train, shape, 10, seed, device),
            SyntheticDataset(n_test, shape, 10, seed + 1, device))
