"""Distributed runtime, flat arenas, DDP, and the multi-rank launcher."""
from . import runtime
from .arena import ParamArena, flatten_module
from .ddp import DDP, DistributedDataParallel
from .runtime import (all_gather_flat, all_reduce, all_reduce_coalesced, barrier, broadcast,
                      destroy_process_group, get_local_rank, get_rank, get_world_size,
                      init_process_group, is_initialized, is_main_process)

__all__ = ["runtime", "ParamArena", "flatten_module", "DDP", "DistributedDataParallel",
           "TensorParallelMLP",
           "init_process_group", "destroy_process_group", "get_rank", "get_world_size",
           "get_local_rank", "is_initialized", "is_main_process", "all_reduce",
           "all_reduce_coalesced", "broadcast", "all_gather_flat", "barrier"]


def __getattr__(name):
    # tensor_parallel builds on nn/ (which imports this package): resolved on first use
    if name == "TensorParallelMLP":
        from .tensor_parallel import TensorParallelMLP

        return TensorParallelMLP
    raise AttributeError(name)
