"""Fault injection for the failure-handling tests.

TDP_FAULT="rank:step" makes that rank raise at that global step (the launcher must then tear
down every other rank); TDP_FAULT="rank:step:stall" makes it hang instead, without exiting, so
the OTHER ranks must detect the dead peer through the collective timeout (gloo's process-group
timeout on CPU, the RCCL watchdog of csrc/comm.h on MI355X; TDP_TIMEOUT_S sets both)."""
from __future__ import annotations

import os
import time


class InjectedFault(RuntimeError):
    pass


def maybe_inject(rank: int, step: int) -> None:
    spec = os.environ.get("TDP_FAULT")
    if not spec:
        return
    parts = spec.split(":")
    r, s = int(parts[0]), int(parts[1])
    if r != rank or s != step:
        return
    if len(parts) > 2 and parts[2] == "stall":
        while True:  # a hung rank: alive, never reaching the next collective
            time.sleep(1.0)
    raise InjectedFault(f"injected fault on rank {rank} at step {step}")
