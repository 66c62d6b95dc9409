"""Where native backward kernels write parameter gradients.

A parameter managed by a :class:`~..parallel.arena.ParamArena` carries ``_tdp_gslot =
(grad_arena, offset)``. When its ``.grad`` is ``None`` (the normal case after
``zero_grad(set_to_none=True)``) the backward kernel writes straight into a *fresh view* of that
slot and returns it; autograd's AccumulateGrad then steals the view as ``.grad`` (no copy), so
the DDP bucket already holds the gradient when the reducer's hook fires -- the reference's
bucket copy-in / copy-out disappears. When ``.grad`` already holds a
value (gradient accumulation, ``no_sync``) a fresh tensor is returned and autograd adds it.
"""
from __future__ import annotations

import torch


def grad_dest(p: torch.Tensor | None) -> torch.Tensor | None:
    if p is None:
        return None
    slot = getattr(p, "_tdp_gslot", None)
    if slot is not None and p.grad is None:
        buf, off = slot
        return buf[off: off + p.numel()].view(p.shape)
    return torch.empty_like(p)


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
