"""Where native backward kernels write parameter gradients.

A parameter managed by a :class:`~..parallel.arena.ParamArena` carries ``_tdp_gslot =
(grad_arena, offset)``. When its ``.grad`` is ``None`` (the normal case after
``zero_grad(set_to_none=True)``) the backward kernel writes straight into a *fresh view* of that
slot and returns it; autograd's AccumulateGrad then steals the view as ``.grad`` (no copy), so
the DDP bucket already holds the gradient when the reducer's hook fires -- the reference's
bucket copy-in / copy-out disappears. When ``.grad`` already holds a
value (gradient accumulation, ``no_sync``) a fresh tensor is returned and autograd adds it.

A parameter used more than once in one forward (a layer applied twice, tied weights) gets the
slot for ONE of its backward GEMMs only: AccumulateGrad runs once, after autograd has summed
every use's gradient, so ``p.grad`` is still None at each use; handing the same slot to two GEMMs
would let the second overwrite the first's partial gradient before the sum. The slot is
therefore given out once per autograd graph task (``torch._C._current_graph_task_id``); later
uses in the same backward get fresh tensors. The optimizer epilogue is disabled for such
parameters (``note_use`` counts uses per DDP iteration, ``DDP.epilogue_slot`` checks them).
"""
from __future__ import annotations

import torch

from ..parallel.arena import slot_view


_task_id = getattr(torch._C, "_current_graph_task_id", lambda: -1)


def grad_dest(p: torch.Tensor | None) -> torch.Tensor | None:
    if p is None:
        return None
    slot = getattr(p, "_tdp_gslot", None)
    if slot is not None and p.grad is None:
        task = _task_id()
        if task < 0 or getattr(p, "_tdp_slot_task", None) != task:
            p._tdp_slot_task = task
            buf, off = slot
            return slot_view(buf, p, off)  # the parameter's own layout (channels_last convs)
    return torch.empty_like(p)


def note_use(p: torch.Tensor | None) -> None:
    """Forward-time use count of a DDP parameter (the optimizer epilogue and the factored
    synchronisation need exactly one)."""
    if p is None:
        return
    ref = getattr(p, "_tdp_epi", None) or getattr(p, "_tdp_factor", None)
    if ref is not None:
        ddp = ref()
        if ddp is not None:
            ddp._note_use(p)


def epilogue_target(p: torch.Tensor | None):
    """``(reducer_backend, arena_offset)`` when the weight-gradient GEMM of ``p`` should apply the
    DDP's fused optimizer in its epilogue instead of storing the gradient (world size 1, fused
    optimizer registered, gradient sync on, ``p.grad`` empty); else None. See
    ``DistributedDataParallel.register_fused_optimizer``."""
    ref = getattr(p, "_tdp_epi", None) if p is not None else None
    if ref is None or p.grad is not None:
        return None
    ddp = ref()
    return ddp.epilogue_slot(p) if ddp is not None else None


def bias_epilogue(b: torch.Tensor | None):
    """``(backend, arena_offset, span)`` when the kernel that reduces the bias gradient of ``b``
    should also apply the fused optimizer to it (``DistributedDataParallel.bias_epilogue``)."""
    ref = getattr(b, "_tdp_epi", None) if b is not None else None
    if ref is None or b.grad is not None:
        return None
    ddp = ref()
    return ddp.bias_epilogue(b) if ddp is not None else None


def hand_off(p: torch.Tensor | None, t: torch.Tensor | None) -> None:
    """``t`` (``p``'s gradient slot) goes to autograd unwritten: a kernel applied the update."""
    ref = getattr(p, "_tdp_epi", None) if p is not None else None
    ddp = ref() if ref is not None else None
    if ddp is not None and t is not None:
        ddp.note_handed(p, t)


def factor_target(p: torch.Tensor | None):
    """The DDP whose factored synchronisation replaces the weight-gradient GEMM of ``p`` in
    this backward (``DistributedDataParallel.factor_slot``), else None."""
    ref = getattr(p, "_tdp_factor", None) if p is not None else None
    if ref is None or p.grad is not None:
        return None
    ddp = ref()
    return ddp.factor_slot(p) if ddp is not None else None


def needs(ctx, i: int) -> bool:
    return bool(ctx.needs_input_grad[i])


class SharedGrad:
    """One gradient buffer shared by the consumers of a forked tensor (:func:`fork`).

    A residual block's input ``x`` feeds the block's first convolution and its identity path;
    autograd would give each consumer its own gradient tensor and add them (one extra
    read-read-write pass over an activation-sized tensor per block). Consumers that know the sink
    instead ``deposit`` into ``buf``: the first one writes it, later ones accumulate into it --
    the input-gradient GEMM with ``beta = 1`` (csrc/gemm_f32_fast.hip epilogue), a strided phase
    with ``copy4d(accumulate=True)`` -- and all return ``buf`` itself, which ``fork``'s backward
    then passes on once."""

    __slots__ = ("buf",)

    def __init__(self):
        self.buf = None

    def deposit(self, g: torch.Tensor) -> torch.Tensor:
        """Generic path (consumers without a fused accumulate): ``buf += g``."""
        if self.buf is None:
            self.buf = g
        else:
            self.buf.add_(g)
        return self.buf


class _Fork(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, sink, n):
        ctx.sink = sink
        return tuple(x.view_as(x) for _ in range(n))

    @staticmethod
    def backward(ctx, *grads):
        sink = ctx.sink
        buf, sink.buf = sink.buf, None
        total = buf
        for g in grads:  # consumers that did not deposit: their gradients are added here
            if g is None or g is buf:
                continue
            total = g if total is None else total.add_(g)
        return total, None, None


def fork(x: torch.Tensor, sink: SharedGrad, n: int = 2):
    """``n`` aliases of ``x`` whose gradients meet in ``sink`` (see :class:`SharedGrad`)."""
    return _Fork.apply(x, sink, n)
