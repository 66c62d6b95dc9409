"""Host relay for the native communicator: W ranks on ONE GPU.

RCCL, like NCCL, refuses two ranks on one device ("Duplicate GPU detected"), and a gpurun box
has one MI355X. ``init_process_group("relay")`` (or ``TDP_GPU_RELAY=1`` with any GPU backend)
keeps every rank on the GPU -- same arenas, same gfx950 kernels, same C++ reducer with its
sharded / factored / replicated updates -- but gives it a ``RelayCommunicator``
(csrc/bindings.cpp) whose collectives call back into :class:`HostRelay`: the device buffers are
copied to the host, reduced / gathered with torch.distributed over gloo, and copied back. It is
a correctness vehicle for the multi-rank device path (tests/test_relay_gpu.py), orders of
magnitude slower than RCCL over xGMI and eager-only (a relayed collective cannot be captured
into a hipGraph).

Semantics match RCCL's: ``avg`` = sum / W; every rank ends with bit-identical results (gloo's
all-reduce computes each element once and distributes it); in-place variants (send buffer
inside the receive buffer) are safe because the send side is read completely first.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

_OPS = {"sum": dist.ReduceOp.SUM, "avg": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX,
        "min": dist.ReduceOp.MIN, "prod": dist.ReduceOp.PRODUCT}


def _host(t: torch.Tensor) -> torch.Tensor:
    """A host copy in a dtype gloo reduces exactly like RCCL does (bf16 / fp16 as float32)."""
    h = t.detach().to("cpu", copy=True)
    return h.float() if h.dtype in (torch.bfloat16, torch.float16) else h


def _back(dst: torch.Tensor, h: torch.Tensor) -> None:
    dst.copy_(h.to(dst.dtype))
    torch.cuda.synchronize(dst.device)


class HostRelay:
    def __init__(self, world: int):
        self.world = world

    # world size 1 (no process group): every collective is a copy
    def _solo(self, send, recv):
        if recv.data_ptr() != send.data_ptr():
            recv.copy_(send)
        torch.cuda.synchronize(recv.device)

    def all_reduce(self, send, recv, op):
        if self.world == 1:
            return self._solo(send, recv)
        h = _host(send)
        dist.all_reduce(h, op=_OPS[op])
        if op == "avg":
            h.div_(self.world)
        _back(recv, h)

    def broadcast(self, buf, root):
        if self.world == 1:
            return None
        h = _host(buf)
        dist.broadcast(h, root)
        _back(buf, h)

    def all_gather(self, send, recv):
        if self.world == 1:
            return self._solo(send, recv)
        h = _host(send)
        parts = [torch.empty_like(h) for _ in range(self.world)]
        dist.all_gather(parts, h)
        _back(recv, torch.cat(parts))

    def reduce_scatter(self, send, recv, op):
        if self.world == 1:
            return self._solo(send, recv)
        h = _host(send)  # the whole send buffer first: recv may alias a slice of it
        dist.all_reduce(h, op=_OPS[op])
        if op == "avg":
            h.div_(self.world)
        n = recv.numel()
        r = dist.get_rank()
        _back(recv, h[r * n: (r + 1) * n])

    def send(self, buf, peer):
        dist.send(_host(buf), peer)

    def recv(self, buf, peer):
        h = _host(buf)
        dist.recv(h, peer)
        _back(buf, h)
