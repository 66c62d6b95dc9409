"""Per-rank seed offsetting (REF/multi-GPU-training-torch.py:54-69).

Reference semantics: s = torch.initial_seed() (random per spawned process), then torch / cuda /
Python / NumPy are seeded with s + rank (NumPy and Python with (s mod 2^32-1) + rank) and the
deterministic-conv flag is set. ``base_seed`` (optional, an addition) makes runs reproducible:
it replaces the per-process random s.
"""
from __future__ import annotations

import random

import numpy as np
import torch


def set_seed_based_on_rank(rank: int, base_seed: int | None = None) -> int:
    s = int(torch.initial_seed()) if base_seed is None else int(base_seed)
    torch.manual_seed(s + rank)
    if torch.cuda.is_available():
        torch.cuda.manual_seed(s + rank)
        torch.backends.cudnn.deterministic = True
    reduced = s % (2 ** 32 - 1)
    random.seed(reduced + rank)
    np.random.seed((reduced + rank) % (2 ** 32))
    return s + rank


def rng_report(device) -> str:
    """The reference's print_rand debug line (REF/multi-GPU-training-torch.py:180-183)."""
    return (f"Dev {device}, Python random state: {random.getstate()[1][:3]}, "
            f"numpy random state: {np.random.get_state()[1][:3]}\n"
            f"Dev {device}, Torch initial_seed: {torch.initial_seed()}")
