"""Distributed runtime: process-group bootstrap and collectives (one process per MI355X).

Reference behaviour (REF/multi-GPU-training-torch.py:29-51):
``setup(rank, world)`` hard-codes MASTER_ADDR/PORT, calls ``init_process_group("nccl")`` (gloo if
NCCL is unavailable) and binds the device *after* the process group; ``cleanup()`` destroys it.

Here ``init_process_group``
  * reads RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT (torchrun, our launcher,
    or explicit arguments);
  * binds ``cuda:local_rank`` BEFORE any communicator exists (SURVEY.md §7.1 order fix);
  * rendezvouses through torch's TCPStore (env://) and a gloo group for host-side control;
  * on GPUs creates the native RCCL communicator (``csrc/comm.cpp``): rank 0's ncclUniqueId is
    published through the same store, every rank calls ncclCommInitRank;
  * also registers torch's own NCCL(=RCCL) backend for cuda tensors (lazily initialised by torch,
    costs nothing unless user code calls ``torch.distributed`` collectives on GPU tensors).
All collectives below take GPU tensors through the native communicator on the current HIP stream
and CPU tensors through gloo.
"""
from __future__ import annotations

import datetime as _dt
import os
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

from .._native import native


@dataclass
class _State:
    initialized: bool = False
    backend: str = "gloo"  # "rccl" | "relay" | "gloo"
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = field(default_factory=lambda: torch.device("cpu"))
    comm: object = None  # native Communicator
    owns_torch_pg: bool = False


_S = _State()


def _env_int(name, default):
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def is_initialized() -> bool:
    return _S.initialized


def get_rank() -> int:
    return _S.rank


def get_world_size() -> int:
    return _S.world


def get_local_rank() -> int:
    return _S.local_rank


def get_backend() -> str:
    return _S.backend


def device() -> torch.device:
    return _S.device


def comm():
    """The native RCCL communicator (None on CPU / gloo)."""
    return _S.comm


def is_main_process() -> bool:
    return _S.rank == 0


def init_process_group(backend: str | None = None, rank: int | None = None,
                       world_size: int | None = None, local_rank: int | None = None,
                       master_addr: str | None = None, master_port: int | None = None,
                       timeout: _dt.timedelta | None = None) -> None:
    """Join the job. ``backend``: "nccl"/"rccl" (GPU), "gloo" (CPU), "relay" (GPU tensors and
    kernels, collectives relayed through the host over gloo: several ranks sharing one GPU,
    parallel/relay.py), "peer" (several ranks sharing one GPU with device-side, capturable
    collectives through IPC-mapped windows, parallel/peer.py) or None (auto).
    ``TDP_GPU_RELAY=1`` / ``TDP_GPU_PEER=1`` turn a GPU backend into "relay" / "peer".

    Auto picks RCCL when a GPU is visible, else gloo (the reference's NCCL-else-gloo rule,
    REF/multi-GPU-training-torch.py:34-42, decided on what can actually run).
    """
    if _S.initialized:
        raise RuntimeError("process group already initialised")
    rank = _env_int("RANK", 0) if rank is None else rank
    world = _env_int("WORLD_SIZE", 1) if world_size is None else world_size
    local_rank = _env_int("LOCAL_RANK", rank) if local_rank is None else local_rank
    os.environ.setdefault("MASTER_ADDR", master_addr or "127.0.0.1")
    if master_addr:
        os.environ["MASTER_ADDR"] = master_addr
    if master_port is not None:
        os.environ["MASTER_PORT"] = str(master_port)
    os.environ.setdefault("MASTER_PORT", "29500")
    want = (backend or "auto").lower()
    gpu_kind = want in ("nccl", "rccl", "auto") and torch.cuda.is_available()
    peer = want == "peer" or (os.environ.get("TDP_GPU_PEER", "0") == "1" and gpu_kind)
    relay = not peer and (want == "relay" or (os.environ.get("TDP_GPU_RELAY", "0") == "1" and
                                              gpu_kind))
    if relay or peer:
        if not torch.cuda.is_available():
            raise RuntimeError(f"backend '{'peer' if peer else 'relay'}' needs a GPU")
        use_gpu = True
    elif want in ("nccl", "rccl"):
        if not torch.cuda.is_available():
            raise RuntimeError("backend 'nccl' (RCCL) requested but no GPU is visible")
        use_gpu = True
    elif want == "gloo":
        use_gpu = False
    elif want == "auto":
        use_gpu = torch.cuda.is_available()
    else:
        raise ValueError(f"unknown backend {backend!r}")

    if use_gpu and peer:
        from .peer import peer_device

        torch.cuda.set_device(peer_device())  # the one-GPU vehicle: every rank on one device
        dev = torch.device("cuda", torch.cuda.current_device())
    elif use_gpu:
        torch.cuda.set_device(local_rank % torch.cuda.device_count())
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    # collective timeout: gloo's PG timeout and the RCCL watchdog (csrc/comm.h) -- TDP_TIMEOUT_S
    # (seconds) or TDP_TIMEOUT_MIN (minutes); defaults: torch's 30 min (gloo) / 10 min (NCCL)
    if timeout is None:
        if os.environ.get("TDP_TIMEOUT_S"):
            timeout = _dt.timedelta(seconds=float(os.environ["TDP_TIMEOUT_S"]))
        else:
            timeout = _dt.timedelta(minutes=float(os.environ.get("TDP_TIMEOUT_MIN", "30")))
    owns = False
    # a single-rank job needs no rendezvous at all (and must not grab MASTER_PORT)
    if world > 1 and not dist.is_initialized():
        pg_backend = "cpu:gloo,cuda:nccl" if use_gpu and not (relay or peer) else "gloo"
        dist.init_process_group(backend=pg_backend, rank=rank, world_size=world, timeout=timeout)
        owns = True
    _S.initialized = True
    _S.backend = ("peer" if peer else "relay" if relay else "rccl") if use_gpu else "gloo"
    _S.rank, _S.world, _S.local_rank, _S.device = rank, world, local_rank, dev
    _S.owns_torch_pg = owns
    if use_gpu and peer:
        from .peer import make_peer_communicator

        _S.comm = make_peer_communicator(rank, world, dev.index)
    elif use_gpu and relay:
        from .relay import HostRelay

        _S.comm = native().RelayCommunicator(rank, world, dev.index, HostRelay(world))
    elif use_gpu:
        C = native()
        if world == 1:
            uid = C.rccl_unique_id()
        else:
            store = dist.distributed_c10d._get_default_store()
            key = "tdp/rccl_uid"
            if rank == 0:
                store.set(key, C.rccl_unique_id())
            uid = store.get(key)
        _S.comm = C.Communicator(uid, rank, world, dev.index)


def destroy_process_group() -> None:
    if not _S.initialized:
        return
    if _S.comm is not None and torch.cuda.is_available():
        torch.cuda.synchronize()
        if _S.backend == "peer" and _S.world > 1 and dist.is_initialized():
            dist.barrier()  # every rank's kernels are done before any window is freed
    _S.comm = None
    if _S.owns_torch_pg and dist.is_initialized():
        dist.destroy_process_group()
    _S.initialized = False
    _S.world, _S.rank = 1, 0


# ------------------------------------------------------------------------------ collectives
def _gpu_path(t: torch.Tensor) -> bool:
    if t.is_cuda:
        if _S.comm is None:
            if _S.world == 1:
                return True
            raise RuntimeError("GPU collective without an RCCL communicator (backend is gloo)")
        return True
    return False


_OPS = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN,
        "prod": dist.ReduceOp.PRODUCT}


def all_reduce(t: torch.Tensor, op: str = "sum") -> torch.Tensor:
    """In-place all-reduce (op: sum|avg|max|min|prod). Ordered on the current stream."""
    if _S.world == 1:
        return t
    if _gpu_path(t):
        _S.comm.all_reduce(t, op)
    else:
        if op == "avg":
            t.div_(_S.world)
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
        else:
            dist.all_reduce(t, op=_OPS[op])
    return t


def all_reduce_coalesced(tensors, op: str = "sum"):
    """One collective per dtype for many small tensors (the reference issues
    5 for its epoch metrics). Tensors are packed in their OWN dtype, so integer counters stay
    exact at any size (no float32 round trip above 2^24)."""
    if _S.world == 1 or not tensors:
        return tensors
    groups = {}
    for t in tensors:
        groups.setdefault((t.dtype, t.device), []).append(t)
    for (dt, dev), ts in groups.items():
        flat = torch.cat([t.reshape(-1) for t in ts])
        all_reduce(flat, op)
        off = 0
        for t in ts:
            n = t.numel()
            t.copy_(flat[off: off + n].view_as(t))
            off += n
    return tensors


def broadcast(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    if _S.world == 1:
        return t
    if _gpu_path(t):
        _S.comm.broadcast(t, src)
    else:
        dist.broadcast(t, src)
    return t


def all_gather_flat(t: torch.Tensor) -> torch.Tensor:
    """Concatenation of every rank's ``t`` (flattened): [world * t.numel()]."""
    if _S.world == 1:
        return t.reshape(-1)
    t = t.contiguous()
    if _gpu_path(t):
        out = torch.empty(_S.world * t.numel(), dtype=t.dtype, device=t.device)
        _S.comm.all_gather(out, t.reshape(-1))
        return out
    parts = [torch.empty_like(t) for _ in range(_S.world)]
    dist.all_gather(parts, t)
    return torch.cat([p.reshape(-1) for p in parts])


def reduce_scatter_flat(t: torch.Tensor, op: str = "sum") -> torch.Tensor:
    if _S.world == 1:
        return t.reshape(-1).clone()
    t = t.contiguous().reshape(-1)
    n = t.numel() // _S.world
    if _gpu_path(t):
        out = torch.empty(n, dtype=t.dtype, device=t.device)
        _S.comm.reduce_scatter(out, t, op)
        return out
    full = t.clone()
    all_reduce(full, op)
    return full[_S.rank * n: (_S.rank + 1) * n].clone()


def barrier() -> None:
    """Block until every rank arrives (reference M7/M9: a 1-element all-reduce on NCCL)."""
    if _S.world == 1:
        if _S.device.type == "cuda":
            torch.cuda.current_stream().synchronize()
        return
    if _S.comm is not None:
        x = torch.ones(1, device=_S.device)
        _S.comm.all_reduce(x, "sum")
        _S.comm.watch_current("barrier")
        _S.comm.synchronize_current()
    else:
        dist.barrier()


class SyncGroup:
    """Collectives SyncBatchNorm needs, over the default group."""

    def all_gather_flat(self, t):
        return all_gather_flat(t)

    def all_reduce_sum_(self, t):
        return all_reduce(t, "sum")


def broadcast_object(obj, src: int = 0):
    if _S.world == 1:
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=src)
    return lst[0]
