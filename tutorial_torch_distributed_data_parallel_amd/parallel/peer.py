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


def peer_device() -> int:
    """The ONE device every rank of the peer vehicle binds to (TDP_PEER_DEVICE, default 0),
    whatever its LOCAL_RANK: the vehicle is defined for ranks that share a GPU."""
    return int(os.environ.get("TDP_PEER_DEVICE", "0"))


def device_key(device: int) -> str:
    """Identity of the physical device behind ``device`` (PCI location when the runtime reports
    it, else the UUID, else the index): equal keys = the same GPU, whatever the visible-device
    mapping of each process."""
    import torch

    pr = torch.cuda.get_device_properties(device)
    bus = getattr(pr, "pci_bus_id", None)
    if bus is not None:
        return f"pci:{getattr(pr, 'pci_domain_id', 0)}:{bus}:{getattr(pr, 'pci_device_id', 0)}"
    uuid = getattr(pr, "uuid", None)
    return f"uuid:{uuid}" if uuid is not None else f"index:{device}"


def require_one_device(keys) -> None:
    """The peer vehicle orders its cross-rank hand-offs with agent-scope release / acquire over
    coarse-grained windows (csrc/peer.hip): valid only while every rank runs on the SAME GPU.
    Ranks on different GPUs would exchange through xGMI with no system-scope ordering -- a
    silently unordered collective -- so such a job is refused."""
    keys = list(keys)
    if len(set(keys)) > 1:
        raise RuntimeError(
            "peer vehicle (TDP_GPU_PEER=1 / backend 'peer'): ranks are on different GPUs "
            f"({', '.join(f'rank {r}: {k}' for r, k in enumerate(keys))}); it is a one-GPU "
            "correctness vehicle whose device-scope ordering does not hold across devices. "
            "Use RCCL (backend 'nccl') for ranks on different GPUs.")


def make_peer_communicator(rank: int, world: int, device: int):
    """Create this rank's window, publish its IPC handle, open every peer's (collective over the
    default store: every rank must call it). Refuses ranks on different GPUs."""
    slot = int(float(os.environ.get("TDP_PEER_SLOT_MB", "64")) * 2 ** 20) // 256 * 256
    if world > 1:
        store = dist.distributed_c10d._get_default_store()
        store.set(f"tdp/peer/dev/{rank}", device_key(device))
        require_one_device(store.get(f"tdp/peer/dev/{p}").decode() for p in range(world))
    comm = native().PeerCommunicator(rank, world, device, slot)
    if world > 1:
        store.set(f"tdp/peer/{rank}", comm.local_handle())
        handles = [store.get(f"tdp/peer/{p}") for p in range(world)]
        comm.connect(handles)
        # nobody may free a window before every peer has opened it (teardown mirrors this)
        dist.barrier()
    else:
        comm.connect([comm.local_handle()])
    return comm
