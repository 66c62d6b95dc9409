"""Accelerate-style facade (Accelerator.prepare / backward / save_model ...)."""
from .accelerator import AcceleratedOptimizer, Accelerator, ShardedLoader

__all__ = ["Accelerator", "AcceleratedOptimizer", "ShardedLoader"]
