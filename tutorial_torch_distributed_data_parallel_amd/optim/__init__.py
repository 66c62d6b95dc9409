"""Fused optimizers (native single-pass kernels on GPU; torch semantics)."""
from .fused import SGD, Adam, AdamW

__all__ = ["SGD", "Adam", "AdamW"]
