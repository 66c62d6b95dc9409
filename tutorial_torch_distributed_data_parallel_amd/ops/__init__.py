"""Differentiable ops over the native gfx950 kernels (CPU tensors use the torch reference)."""
from .linear import linear
from .loss import count_correct, cross_entropy
from .norm import batch_norm

__all__ = ["linear", "cross_entropy", "count_correct", "batch_norm"]
