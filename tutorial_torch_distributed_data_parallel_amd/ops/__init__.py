"""Differentiable ops over the native gfx950 kernels (CPU tensors use the torch reference)."""
from .conv import conv2d
from .linear import linear
from .loss import backward, count_correct, cross_entropy, linear_cross_entropy, seed_grad
from .norm import batch_norm
from .pool import adaptive_avg_pool2d, add_relu, dropout, flatten, max_pool2d

__all__ = ["linear", "conv2d", "max_pool2d", "adaptive_avg_pool2d", "dropout", "add_relu",
           "cross_entropy", "linear_cross_entropy", "count_correct", "batch_norm", "backward", "seed_grad", "flatten"]
