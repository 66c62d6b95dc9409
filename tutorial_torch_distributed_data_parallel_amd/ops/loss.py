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


_TICKETS: dict = {}


def _ticket(device) -> torch.Tensor:
    """Zeroed int32 ticket words per (device, stream) for head_ce's last-arriver hand-off (the
    kernel leaves them zero again; one stream's launches never overlap)."""
    key = (device, torch.cuda.current_stream(device).cuda_stream)
    t = _TICKETS.get(key)
    if t is None:
        t = torch.zeros(16, dtype=torch.int32, device=device)
        _TICKETS[key] = t
    return t


class _LinearCrossEntropyFn(torch.autograd.Function):
    """``cross_entropy(x W^T + b, target)`` for a classifier head (out <= 16, batch <= 256): the
    head GEMM, the loss, the logits gradient for a unit seed and the head's input gradient (gated
    by the previous ReLU, with its bf16 planes) in ONE forward launch (csrc/gemm_skinny.hip
    head_ce); the backward reduces only dW / db (head_bwd with no dx; with the optimizer in its
    epilogue at world size 1). Bit-identical to ``cross_entropy(linear(x, W, b), target)``: the
    same per-row arithmetic in the same order (tests/test_head_ce_gpu.py)."""

    @staticmethod
    def forward(ctx, x2, weight, bias, target, ignore_index, smoothing, mean, acc, gate_in, prev):
        from .linear import planes_input_fit

        C = native()
        train = ctx.needs_input_grad[0] or ctx.needs_input_grad[1] or ctx.needs_input_grad[2]
        gate = x2 if gate_in else None
        want_dx = bool(ctx.needs_input_grad[0])
        out = C.head_ce(x2, weight, bias, target, ignore_index, smoothing, mean, acc,
                        with_grad=bool(train), gate=gate if want_dx else None,
                        planes=want_dx and planes_input_fit(x2.shape[0], x2.shape[1]),
                        ticket=_ticket(x2.device))
        if not out:
            raise RuntimeError("linear_cross_entropy: head_ce refused the operands")
        loss, lse, logits = out[0], out[1], out[2]
        ctx.pre = (out[3], out[4] if want_dx else None,
                   out[5] if want_dx and out[5].numel() else None) if train else None
        ctx.cfg = (ignore_index, smoothing, mean)
        ctx.gate_in = gate_in
        ctx.prev_w = prev[0] if prev else None
        ctx.params = (weight, bias)
        ctx.save_for_backward(x2, weight, target, lse, logits)
        return loss

    @staticmethod
    def backward(ctx, gout):
        from ._grad import bias_epilogue, epilogue_target, grad_dest, hand_off, needs
        from .linear import _mark_gated, _prefetch_prev_g, _tp_epilogue, attach_planes

        C = native()
        x2, weight, target, lse, logits = ctx.saved_tensors
        w_param, b_param = ctx.params
        pre, ctx.pre = ctx.pre, None
        ignore_index, smoothing, mean = ctx.cfg
        gate = x2 if ctx.gate_in else None
        if pre is not None and _is_unit_seed(gout):
            g, dx, pl = pre
        else:  # a scaled / accumulated upstream gradient: the unfused path
            g = C.ce_bwd(logits, target, lse, gout.reshape(1).float(), ignore_index, smoothing,
                         mean)
            dx = pl = None
        want_dx, want_w = needs(ctx, 0), needs(ctx, 1)
        db = grad_dest(b_param) if b_param is not None and needs(ctx, 2) else None
        dw = grad_dest(w_param) if want_w else None
        if dx is None and want_dx:
            dx = torch.empty_like(x2)
            fresh_dx = True
        else:
            fresh_dx = False
        if want_w:
            kw = {}
            epi = epilogue_target(w_param)
            if epi is not None and dw.is_contiguous() and not _tp_epilogue(epi):
                kw = dict(backend=epi[0], w_offset=epi[1])
                be = bias_epilogue(b_param) if db is not None else None
                if be is not None:
                    kw.update(b_offset=be[1], b_span=be[2])
            from .linear import planes_input_fit

            ok, pl2 = C.head_bwd(g, x2, weight, dx if fresh_dx else None, dw, db=db, gate=gate,
                                 planes=fresh_dx and planes_input_fit(x2.shape[0], x2.shape[1]),
                                 **kw)
            if not ok:
                raise RuntimeError("linear_cross_entropy: head_bwd refused the shapes head_ce took")
            if kw:
                hand_off(w_param, dw)
                if "b_offset" in kw:
                    hand_off(b_param, db)
            if fresh_dx:
                pl = pl2
        else:
            if want_dx and fresh_dx:
                dx.copy_(g @ weight)
                if gate is not None:
                    dx.mul_(gate > 0)
            if db is not None:
                db.copy_(g.sum(0))
        if want_dx:
            if gate is not None:
                _mark_gated(dx, x2)
                prev = _prefetch_prev_g(ctx, dx)
                if prev is not None:
                    prev.factor_flush()
            if pl is not None:
                attach_planes(dx, pl)
        return dx, dw, db, None, None, None, None, None, None, None


def linear_cross_entropy(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None,
                         target: torch.Tensor, ignore_index: int = -100,
                         label_smoothing: float = 0.0, reduction: str = "mean",
                         acc: torch.Tensor | None = None) -> torch.Tensor:
    """``cross_entropy(x @ weight.T + bias, target)`` -- a classifier head and its loss (the
    reference's ``criterion(model(inputs), labels)`` for the last Linear,
    REF/multi-GPU-training-torch.py:121-122) -- fused into one launch on MI355X when the head is
    small (out <= 16, batch <= 256, fp32); otherwise (and on CPU) exactly the two ops."""
    from .linear import _factor_owner, linear
    from ._grad import note_use

    fits = (x.is_cuda and x.dim() == 2 and x.dtype == torch.float32 and weight.shape[0] <= 16 and
            x.shape[0] <= 256 and x.shape[1] % 4 == 0 and reduction in ("mean", "sum") and
            weight.stride(1) == 1 and weight.stride(0) % 4 == 0 and weight.data_ptr() % 16 == 0 and
            x.stride(1) == 1 and x.stride(0) % 4 == 0 and x.data_ptr() % 16 == 0 and
            target.dim() == 1 and _factor_owner(weight) is None)
    if not fits:
        return cross_entropy(linear(x, weight, bias), target, ignore_index, label_smoothing,
                             reduction, acc)
    gate_in = bool(getattr(x, "_tdp_relu_out", False))
    if torch.is_grad_enabled():
        note_use(weight)
    pw = getattr(x, "_tdp_prod_w", None) if gate_in else None
    return _LinearCrossEntropyFn.apply(x, weight, bias, target.contiguous().long(),
                                       int(ignore_index), float(label_smoothing),
                                       reduction == "mean", acc, gate_in,
                                       (pw,) if pw is not None else None)


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
