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
    """Forward-time use count of a DDP parameter (the optimizer epilogue needs exactly one)."""
    ref = getattr(p, "_tdp_epi", None) if p is not None else None
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


def needs(ctx, i: int) -> bool:
    return bool(ctx.needs_input_grad[i])
