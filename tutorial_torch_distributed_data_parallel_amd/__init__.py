"""MI355X-native single-node data-parallel training framework.

Capabilities of annalena-k/tutorial-torch-distributed-data-parallel, built
MI355X-first: hand-written gfx950 HIP kernels (MFMA GEMM with fused epilogues, fused
cross-entropy, single-pass SGD/Adam, batch-norm/SyncBN), a C++ RCCL communicator and gradient
reducer over a flat gradient arena, DistributedSampler-exact sharding, a 1-8 rank launcher, an
Accelerate-style facade and reference-compatible checkpoints.
"""
from . import data, models, nn, ops, optim, parallel
from ._native import available as native_available
from .parallel import (DDP, DistributedDataParallel, barrier, destroy_process_group,
                       get_rank, get_world_size, init_process_group)

__version__ = "0.1.0"
__all__ = ["data", "models", "nn", "ops", "optim", "parallel", "DDP",
           "DistributedDataParallel", "init_process_group", "destroy_process_group", "barrier",
           "get_rank", "get_world_size", "native_available"]
