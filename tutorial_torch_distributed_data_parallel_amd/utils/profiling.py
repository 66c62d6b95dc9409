"""Tracing hooks: roctx ranges (visible in rocprofv3 --marker-trace), RCCL debug passthrough.

The reference only carries commented NCCL_DEBUG lines (REF/multi-GPU-training-torch.py:8-10,
SURVEY.md §5.1). ``range("forward")`` pushes a roctx range through torch's binding when
available (no-op otherwise); ``enable_rccl_debug`` sets NCCL_DEBUG/NCCL_DEBUG_SUBSYS (RCCL reads
the NCCL_* names) before the communicator is created.
"""
from __future__ import annotations

import contextlib
import os

import torch


def enable_rccl_debug(level: str = "INFO", subsys: str | None = "COLL") -> None:
    os.environ["NCCL_DEBUG"] = level
    if subsys:
        os.environ["NCCL_DEBUG_SUBSYS"] = subsys


_ENABLED = os.environ.get("TDP_ROCTX", "0") == "1"


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors nvtx/roctx naming
    if not _ENABLED or not torch.cuda.is_available():
        yield
        return
    try:
        torch.cuda.nvtx.range_push(name)  # routed to roctx on ROCm builds
        pushed = True
    except Exception:
        pushed = False
    try:
        yield
    finally:
        if pushed:
            torch.cuda.nvtx.range_pop()
