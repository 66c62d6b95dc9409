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


def needs(ctx, i: int) -> bool:
    return bool(ctx.needs_input_grad[i])
