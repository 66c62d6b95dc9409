"""Cross-entropy on the fused native kernels.

``acc`` is an optional device accumulator ``[loss_sum, correct, count]`` updated inside the
forward kernel, which is how the training/eval loops keep the reference's per-epoch metric sums
(REF/multi-GPU-training-torch.py:131,147-151) without a host sync per step.
"""
from __future__ import annotations


import torch
import torch.nn.functional as F

from .._native import native


# small heads (the toy MLP's / AlexNet's 128 x 10): the forward kernel also writes the gradient
# for an upstream gradient of 1, so a backward seeded with the cached unit seed (seed_grad /
# backward below; autograd hands the seed tensor itself to this node) launches nothing
_FUSED_GRAD_MAX = 1 << 16


class _CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, ignore_index: int, smoothing: float, mean: bool, acc):
        C = native()
        fused = ctx.needs_input_grad[0] and logits.numel() <= _FUSED_GRAD_MAX
        out = C.ce_fwd(logits, target, ignore_index, smoothing, mean, acc, with_grad=fused)
        loss, lse = out[0], out[1]
        ctx.dpre = out[2] if fused else None
        ctx.save_for_backward(logits, target, lse)
        ctx.cfg = (ignore_index, smoothing, mean)
        return loss

    @staticmethod
    def backward(ctx, gout):
        dpre, ctx.dpre = ctx.dpre, None
        if dpre is not None and _is_unit_seed(gout):
            return dpre, None, None, None, None, None
        logits, target, lse = ctx.saved_tensors
        ignore_index, smoothing, mean = ctx.cfg
        d = native().ce_bwd(logits, target, lse, gout.reshape(1).float(), ignore_index, smoothing,
                            mean)
        return d, None, None, None, None, None


def cross_entropy(logits: torch.Tensor, target: torch.Tensor, ignore_index: int = -100,
                  label_smoothing: float = 0.0, reduction: str = "mean",
                  acc: torch.Tensor | None = None) -> torch.Tensor:
    if not logits.is_cuda:
        loss = F.cross_entropy(logits, target, ignore_index=ignore_index,
                               label_smoothing=label_smoothing, reduction=reduction)
        if acc is not None:
            with torch.no_grad():
                valid = target != ignore_index
                per = F.cross_entropy(logits.detach(), target, ignore_index=ignore_index,
                                      label_smoothing=label_smoothing, reduction="sum")
                acc[0] += per
                acc[1] += ((logits.argmax(1) == target) & valid).sum()
                acc[2] += valid.sum()
        return loss
    if reduction not in ("mean", "sum"):
        raise NotImplementedError("native cross_entropy supports reduction='mean'|'sum'")
    if logits.dim() != 2:
        raise ValueError("native cross_entropy expects [batch, classes] logits")
    if logits.stride(1) != 1:
        logits = logits.contiguous()
    return _CrossEntropyFn.apply(logits, target.contiguous().long(), int(ignore_index),
                                 float(label_smoothing), reduction == "mean", acc)


_SEEDS: dict = {}


def seed_grad(loss: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
    """The gradient that seeds ``loss.backward``: a cached device tensor of ``scale`` (no
    ``ones_like`` fill kernel per step -- what autograd launches when no gradient is passed --
    and no ATen division for ``loss / accumulation_steps``). Read-only by contract: the native
    backward kernels only read it."""
    key = (loss.device, loss.dtype, tuple(loss.shape), float(scale))
    g = _SEEDS.get(key)
    if g is None:
        g = torch.full(loss.shape, float(scale), device=loss.device, dtype=loss.dtype)
        _SEEDS[key] = g
    return g


def _is_unit_seed(g: torch.Tensor) -> bool:
    """``g`` is one of the cached seeds of value 1 (read-only by contract, so still 1)."""
    for key, t in _SEEDS.items():
        if t is g:
            return key[3] == 1.0
    return False


def backward(loss: torch.Tensor, scale: float = 1.0, **kwargs) -> None:
    """``(loss * scale).backward(**kwargs)`` without the seed-gradient fill / scaling kernels."""
    loss.backward(seed_grad(loss, scale), **kwargs)


@torch.no_grad()
def count_correct(logits: torch.Tensor, target: torch.Tensor, acc: torch.Tensor) -> None:
    """acc[1] += #(argmax == target), acc[2] += #rows (fused argmax+compare+count)."""
    if not logits.is_cuda:
        acc[1] += (logits.argmax(1) == target).sum()
        acc[2] += target.numel()
        return
    native().count_correct(logits.contiguous(), target.contiguous().long(), acc)
