"""Fault injection for the fail-fast tests: TDP_FAULT="rank:step" makes that
rank raise at that global step; the launcher must then tear down every other rank."""
from __future__ import annotations

import os


class InjectedFault(RuntimeError):
    pass


def maybe_inject(rank: int, step: int) -> None:
    spec = os.environ.get("TDP_FAULT")
    if not spec:
        return
    r, s = (int(v) for v in spec.split(":"))
    if r == rank and s == step:
        raise InjectedFault(f"injected fault on rank {rank} at step {step}")
