"""Samplers with the reference's sharding semantics and on-device synthetic data."""
from .sampler import BatchShardSampler, DistributedSampler
from .synthetic import DeviceLoader, SyntheticDataset, cifar_like

__all__ = ["DistributedSampler", "BatchShardSampler", "SyntheticDataset", "DeviceLoader",
           "cifar_like"]
