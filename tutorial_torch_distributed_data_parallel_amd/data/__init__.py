"""Samplers with the reference's sharding semantics, on-device synthetic data and the host-dataset
pipeline (native prefetcher + on-device resize / flip / normalise)."""
from .host import (CIFAR_MEAN, CIFAR_STD, HostImageDataset, ImageTransform, PrefetchLoader,
                   cifar_like_uint8, load_cifar10_bin, write_cifar10_bin)
from .sampler import BatchShardSampler, DistributedSampler
from .synthetic import DeviceLoader, SyntheticDataset, cifar_like

__all__ = ["DistributedSampler", "BatchShardSampler", "SyntheticDataset", "DeviceLoader",
           "cifar_like", "HostImageDataset", "ImageTransform", "PrefetchLoader",
           "cifar_like_uint8", "load_cifar10_bin", "write_cifar10_bin", "CIFAR_MEAN",
           "CIFAR_STD"]
