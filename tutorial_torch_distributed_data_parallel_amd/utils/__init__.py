"""Seeds, checkpoints, YAML settings, device-side metrics, tracing, fault injection."""
from . import checkpoint, config, fault, metrics, profiling, seed
from .checkpoint import (load_checkpoint, save_ddp_checkpoint, save_model_safetensors,
                         save_training_state, load_training_state)
from .seed import set_seed_based_on_rank

__all__ = ["checkpoint", "config", "fault", "metrics", "profiling", "seed",
           "set_seed_based_on_rank", "save_ddp_checkpoint", "load_checkpoint",
           "save_model_safetensors", "save_training_state", "load_training_state"]
