"""Host-dataset input pipeline (the reference's CIFAR-10 + torchvision transforms + DataLoader).

Reference (REF/data_and_toy_model.py:8-38, REF/multi-GPU-training-torch.py:86-99): CIFAR-10 as
PIL uint8 32x32 images, ``Resize(224) -> RandomHorizontalFlip -> ToTensor -> Normalize(mean,
std)`` per sample in 2 DataLoader worker processes per rank, ``pin_memory=True``, then a 77 MB
float32 H2D copy per 128-sample batch.

Here:
  * ``HostImageDataset`` keeps the samples as ONE uint8 ``[n, H, W, C]`` host tensor (or a
    ``numpy.memmap`` of one) -- 150 MB for the whole CIFAR-10 training set;
  * ``PrefetchLoader`` hands the sampler's epoch order to the native ``HostBatchLoader``
    (csrc/loader.h): C++ worker threads gather the sampled rows into pinned staging slots
    ``depth`` batches ahead, with per-sample flip bits from a counter-based hash of
    (seed, epoch, position);
  * per step one async H2D copy of the uint8 batch (393 KB at 32x32, 200x less than the
    reference's float batch) on the current stream, then ``image_transform`` (csrc/image.hip)
    does resize + flip + /255 + normalise in one pass on the GPU and writes the channels_last
    float batch the convolutions consume.
On CPU the same classes run the torch reference implementation of the transform (the oracle of
the tests). Parity with torchvision/PIL itself is unpinned here (neither is importable): the
kernel implements PIL's upsampling filter (bilinear, half-pixel centres) with PIL-style rounding
to uint8, checked against ``F.interpolate(mode="bilinear", align_corners=False)``.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from .._native import native

# REF/data_and_toy_model.py:17-20 (CIFAR-10 per-channel mean / std)
CIFAR_MEAN = (0.4914, 0.4822, 0.4465)
CIFAR_STD = (0.2023, 0.1994, 0.2010)


class HostImageDataset:
    """uint8 images ``[n, H, W, C]`` + int64 labels, in host memory."""

    def __init__(self, images, labels):
        if isinstance(images, np.ndarray):
            images = torch.from_numpy(np.ascontiguousarray(images))
        if isinstance(labels, np.ndarray):
            labels = torch.from_numpy(labels.astype(np.int64))
        if images.dtype != torch.uint8 or images.dim() != 4:
            raise TypeError("HostImageDataset expects uint8 [n, H, W, C] images")
        self.images = images.contiguous()
        self.labels = labels.to(torch.int64).contiguous()
        if len(self.images) != len(self.labels):
            raise ValueError("images / labels length mismatch")

    def __len__(self):
        return len(self.images)

    def __getitem__(self, i):
        return self.images[i], self.labels[i]

    @property
    def hwc(self):
        return tuple(self.images.shape[1:])


def cifar_like_uint8(n: int = 50000, hw: int = 32, num_classes: int = 10, seed: int = 0):
    """Synthetic CIFAR-10-layout data (no network): uint8 32x32x3 images whose per-class mean
    colour differs, so a model can learn the labels."""
    g = torch.Generator().manual_seed(seed)
    labels = torch.randint(0, num_classes, (n,), generator=g)
    base = torch.randint(40, 216, (num_classes, 1, 1, 3), generator=g).float()
    noise = torch.randn(n, hw, hw, 3, generator=g) * 40.0
    img = (base[labels] + noise).clamp_(0, 255).round_().to(torch.uint8)
    return HostImageDataset(img, labels)


CIFAR10_TRAIN_FILES = tuple(f"data_batch_{i}.bin" for i in range(1, 6))
CIFAR10_TEST_FILES = ("test_batch.bin",)
_CIFAR_RECORD = 1 + 3 * 32 * 32  # label byte + R, G, B planes of 32x32, row-major


def _cifar_dir(root: str) -> str:
    """``root`` itself or the ``cifar-10-batches-bin`` directory the binary archive unpacks to
    (torchvision's CIFAR10(root=...) layout, REF/data_and_toy_model.py:31-36)."""
    import os

    for d in (root, os.path.join(root, "cifar-10-batches-bin")):
        if os.path.isfile(os.path.join(d, "test_batch.bin")) or \
                os.path.isfile(os.path.join(d, "data_batch_1.bin")):
            return d
    raise FileNotFoundError(
        f"no CIFAR-10 binary batches (data_batch_1.bin ... / test_batch.bin) under {root!r} or "
        f"{root!r}/cifar-10-batches-bin: there is no download here -- place the binary archive's "
        "files there (the python-pickle archive is not read: loading pickles executes code)")


def load_cifar10_bin(root: str = "./data", train: bool = True) -> HostImageDataset:
    """CIFAR-10 from its binary distribution: every record is 1 label byte followed by 3072
    bytes (R, G, B planes of 32x32). The files are memory-mapped (no pickle, nothing executed)
    and transposed once to the uint8 [n, 32, 32, 3] layout the native prefetcher gathers from
    (150 MB for the training set)."""
    import os

    d = _cifar_dir(root)
    names = CIFAR10_TRAIN_FILES if train else CIFAR10_TEST_FILES
    imgs, labels = [], []
    for name in names:
        path = os.path.join(d, name)
        raw = np.memmap(path, dtype=np.uint8, mode="r")
        if raw.size % _CIFAR_RECORD:
            raise ValueError(f"{path}: {raw.size} bytes is not a whole number of "
                             f"{_CIFAR_RECORD}-byte CIFAR-10 records")
        rec = raw.reshape(-1, _CIFAR_RECORD)
        labels.append(np.asarray(rec[:, 0], dtype=np.int64))
        imgs.append(np.asarray(rec[:, 1:]).reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1))
        del raw, rec
    if not imgs:
        raise FileNotFoundError(f"no CIFAR-10 files in {d}")
    lab = np.concatenate(labels)
    if lab.size and (lab.min() < 0 or lab.max() > 9):
        raise ValueError("CIFAR-10 labels must be in [0, 9]")
    return HostImageDataset(np.ascontiguousarray(np.concatenate(imgs)), lab)


def write_cifar10_bin(path: str, images: torch.Tensor, labels: torch.Tensor) -> None:
    """Write uint8 [n, 32, 32, 3] images + labels in the CIFAR-10 binary record layout (test
    fixtures, and converting other sources to what load_cifar10_bin reads)."""
    x = images.to(torch.uint8).permute(0, 3, 1, 2).reshape(len(images), -1).numpy()
    rec = np.concatenate([labels.to(torch.uint8).numpy().reshape(-1, 1), x], axis=1)
    rec.astype(np.uint8).tofile(path)


def reference_transform(x_u8: torch.Tensor, flip: torch.Tensor | None, size, mean, std,
                        round_u8: bool = True) -> torch.Tensor:
    """torch implementation of image_transform (CPU path and test oracle); [B,H,W,C] uint8 ->
    [B,C,Ho,Wo] float32."""
    x = x_u8.permute(0, 3, 1, 2).float()
    y = F.interpolate(x, size=tuple(size), mode="bilinear", align_corners=False)
    if round_u8:
        y = y.round()
    if flip is not None:
        y = torch.where(flip.bool().view(-1, 1, 1, 1), y.flip(-1), y)
    m = torch.tensor(mean, dtype=torch.float32, device=y.device).view(1, -1, 1, 1)
    s = torch.tensor(std, dtype=torch.float32, device=y.device).view(1, -1, 1, 1)
    return (y / 255.0 - m) / s


class ImageTransform:
    """Resize(size) + RandomHorizontalFlip(flip_p) + ToTensor + Normalize(mean, std)."""

    def __init__(self, size=224, flip_p: float = 0.5, mean=CIFAR_MEAN, std=CIFAR_STD,
                 round_u8: bool = True, channels_last: bool = True):
        self.size = (size, size) if isinstance(size, int) else tuple(size)
        self.flip_p, self.mean, self.std = float(flip_p), tuple(mean), tuple(std)
        self.round_u8, self.channels_last = round_u8, channels_last

    def __call__(self, x_u8: torch.Tensor, flip: torch.Tensor | None) -> torch.Tensor:
        if x_u8.is_cuda:
            return native().image_transform(x_u8, flip if self.flip_p > 0 else None,
                                            self.size[0], self.size[1], list(self.mean),
                                            list(self.std), self.round_u8, self.channels_last)
        y = reference_transform(x_u8, flip if self.flip_p > 0 else None, self.size, self.mean,
                                self.std, self.round_u8)
        return y.contiguous(memory_format=torch.channels_last) if self.channels_last else y


def _epoch_seed(seed: int, epoch: int) -> int:
    return (int(seed) * 1000003 + int(epoch) * 7919 + 12345) & 0xFFFFFFFFFFFF


class PrefetchLoader:
    """DataLoader for a HostImageDataset: (inputs, labels) device batches in sampler order.

    ``sampler`` (e.g. DistributedSampler) is re-iterated every epoch, so ``set_epoch`` works as
    with torch's DataLoader; the flip bits change with the sampler's epoch (or with every pass
    when the sampler has none)."""

    def __init__(self, dataset: HostImageDataset, batch_size: int, sampler=None,
                 drop_last: bool = False, transform: ImageTransform | None = None, device=None,
                 depth: int = 4, threads: int = 2, seed: int = 0):
        self.dataset, self.batch_size, self.sampler = dataset, batch_size, sampler
        self.drop_last = drop_last
        self.transform = transform or ImageTransform()
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.seed = seed
        self._passes = 0
        self._native = native().HostBatchLoader(dataset.images.reshape(len(dataset), -1),
                                                dataset.labels, batch_size, depth=depth,
                                                threads=threads,
                                                pinned=self.device.type == "cuda")

    def __len__(self):
        n = len(self.sampler) if self.sampler is not None else len(self.dataset)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def __iter__(self):
        idx = list(self.sampler) if self.sampler is not None else list(range(len(self.dataset)))
        epoch = getattr(self.sampler, "epoch", None)
        epoch = self._passes if epoch is None else epoch
        self._passes += 1
        self._native.start_epoch(idx, self.drop_last, _epoch_seed(self.seed, epoch),
                                 self.transform.flip_p)
        h, w, c = self.dataset.hwc
        dev = str(self.device)
        while True:
            out = self._native.next(dev)
            if out is None:
                return
            xu8, y, flip = out
            yield self.transform(xu8.view(-1, h, w, c), flip), y
