"""Gradient clipping (the reference README's pitfall, REF/README.md:92-95).

``clip_grad_norm_`` is ``torch.nn.utils.clip_grad_norm_`` (L2 norm, coefficient
``max_norm / (total_norm + 1e-6)`` clamped to 1) with the whole computation on the MI355X: a
deterministic two-pass sum of squares per gradient (csrc/optim.hip ``sumsq_ranges``), the
coefficient computed on the device and one scaling pass -- no host synchronisation, so it can sit
inside a captured hipGraph step. It returns the total norm as a 0-d device tensor, like torch.

With DDP the two standard placements are:
  * after ``backward()`` (clip the AVERAGED gradient): call this on ``ddp.parameters()``, or with
    a fused optimizer pass ``clip_grad_norm=`` to ``DDP.register_fused_optimizer`` (the norm is
    reduced inside the reduction, before the update);
  * before aggregation (the README's advice: one rank's bad gradient must not spoil the
    average): ``DDP.clip_grad_norm_before_aggregation(max_norm)``.
"""
from __future__ import annotations

import torch

from .._native import native

_BLOCKS = {}  # device -> hyper block used as the norm workspace


def _block(dev: torch.device) -> torch.Tensor:
    blk = _BLOCKS.get(dev)
    if blk is None:
        from ..optim.fused import hyper_slots

        blk = torch.zeros(hyper_slots()["size"], device=dev)
        _BLOCKS[dev] = blk
    return blk


def clip_grad_norm_(parameters, max_norm: float, norm_type: float = 2.0,
                    error_if_nonfinite: bool = False) -> torch.Tensor:
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    params = [p for p in parameters if p.grad is not None]
    for p in params:
        ref = getattr(p, "_tdp_arena", None)
        ddp = getattr(p, "_tdp_fused_owner", None)
        if ref is not None and ddp is not None and ddp() is not None:
            raise RuntimeError(
                "clip_grad_norm_: these gradients belong to a DDP model whose fused optimizer "
                "already applied the update inside the reduction (p.grad is partial there); "
                "pass clip_grad_norm= to DDP.register_fused_optimizer instead")
    if not params:
        return torch.tensor(0.0)
    if (norm_type != 2.0 or not params[0].is_cuda or
            any(p.grad.dtype != torch.float32 or not p.grad.is_contiguous() for p in params)):
        return torch.nn.utils.clip_grad_norm_(params, max_norm, norm_type, error_if_nonfinite)
    from ..optim.fused import hyper_slots

    dev = params[0].grad.device
    blk = _block(dev)
    # parameters of one flat arena: ONE range over the arena gradient instead of one per tensor
    arena = getattr(params[0], "_tdp_arena", None)
    grads = [p.grad for p in params]
    if arena is not None and len(params) == len(arena.params) and \
            all(arena.is_arena_grad(i) for i in range(len(arena.params))):
        grads = [arena.grad]
    native().clip_grad_norm(grads, blk, float(max_norm))
    total = blk[hyper_slots()["norm"]].clone()
    if error_if_nonfinite and not bool(torch.isfinite(total)):
        raise RuntimeError(f"The total norm of order {norm_type} for gradients is non-finite")
    return total
