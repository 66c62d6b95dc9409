"""Peer-memory communicator bootstrap: W ranks on ONE GPU with capture-capable collectives.

``init_process_group("peer")`` (or ``TDP_GPU_PEER=1`` with a GPU backend) gives every rank a
``PeerCommunicator`` (csrc/peer.hip): each rank exports one device window with a HIP IPC handle,
the handles travel through the rendezvous store, and every collective is a single gfx950 kernel
that copies / reduces through the peers' windows, synchronised by device-side counters with
bounded spins. Unlike the host relay (parallel/relay.py) nothing leaves the device and nothing
needs the host, so the multi-rank training step -- bucket collectives on the side stream,
factored gathers, fork / join edges -- is captured into a hipGraph and replayed with real peers
(tests/test_peer_gpu.py). It is a correctness vehicle for one GPU: RCCL over xGMI stays the
transport of a real node.

Semantics match RCCL's: ``avg`` = sum / W; reductions combine the peers in rank order, so every
rank ends with bit-identical results; in-place variants are safe.

Environment: TDP_PEER_SLOT_MB (per-rank staging slot, default 64 MiB; larger collectives are
chunked), TDP_PEER_TIMEOUT_S (bound of every device-side wait, default 30 s).
"""
from __future__ import annotations

import os

import torch.distributed as dist

from .._native import native


def make_peer_communicator(rank: int, world: int, device: int):
    """Create this rank's window, publish its IPC handle, open every peer's (collective over the
    default store: every rank must call it)."""
    slot = int(float(os.environ.get("TDP_PEER_SLOT_MB", "64")) * 2 ** 20) // 256 * 256
    comm = native().PeerCommunicator(rank, world, device, slot)
    if world > 1:
        store = dist.distributed_c10d._get_default_store()
        store.set(f"tdp/peer/{rank}", comm.local_handle())
        handles = [store.get(f"tdp/peer/{p}") for p in range(world)]
        comm.connect(handles)
        # nobody may free a window before every peer has opened it (teardown mirrors this)
        dist.barrier()
    else:
        comm.connect([comm.local_handle()])
    return comm
