"""Flat parameter / gradient arenas.

Every trainable parameter of a model becomes a view into ONE contiguous fp32 buffer, laid out in
*backward order* (reverse registration order, the order autograd produces gradients for
sequential models; torch DDP reaches a similar layout only after rebuilding its buckets at
iteration 1, TORCH/nn/parallel/distributed.py:1199-1229). A second buffer of the same layout
holds the gradients. Consequences, all MI355X-motivated:
  * DDP buckets are contiguous ranges of the gradient arena -> zero-copy all-reduce;
  * the rank-0 weight broadcast of the DDP constructor is ONE collective;
  * the optimizer step is ONE kernel over the whole arena (csrc/optim.hip);
  * a 57M-parameter model is 218 MiB: trivially resident in 288 GB of HBM3E.
Each parameter start is aligned to 64 elements (256 B) so every view is 16-B aligned for the
vectorised kernels; the gaps stay zero in both arenas.
"""
from __future__ import annotations

import torch

ALIGN = 64


def _round_up(n: int, a: int) -> int:
    return (n + a - 1) // a * a


def _cl(p) -> bool:
    """A 4-D parameter in channels_last memory (conv weights: [Cout][R][S][C])."""
    return p.dim() == 4 and not p.is_contiguous() and \
        p.is_contiguous(memory_format=torch.channels_last)


def slot_view(buf: torch.Tensor, p, off: int) -> torch.Tensor:
    """``p``-shaped view of ``buf[off: off + p.numel()]`` with ``p``'s memory layout (contiguous,
    or channels_last for conv weights) -- arena parameter / gradient / optimizer-state slots."""
    if _cl(p):
        C, H, W = p.shape[1], p.shape[2], p.shape[3]
        return buf.as_strided(p.shape, (H * W * C, 1, W * C, C), off)
    return buf[off: off + p.numel()].view(p.shape)


class ParamArena:
    def __init__(self, params, device=None, dtype=torch.float32):
        params = list(params)
        seen, uniq = set(), []
        for p in params:
            if id(p) not in seen:
                seen.add(id(p))
                uniq.append(p)
        self.params = uniq
        if not uniq:
            raise ValueError("ParamArena needs at least one parameter")
        device = torch.device(device) if device is not None else uniq[0].device
        for p in uniq:
            if p.dtype != dtype:
                raise TypeError(f"arena dtype is {dtype}, parameter has {p.dtype}")
        self.offsets, self.numels = [], []
        off = 0
        for p in uniq:
            self.offsets.append(off)
            self.numels.append(p.numel())
            off = _round_up(off + p.numel(), ALIGN)
        self.numel = max(off, ALIGN)
        self.device, self.dtype = device, dtype
        self.data = torch.zeros(self.numel, device=device, dtype=dtype)
        self.grad = torch.zeros(self.numel, device=device, dtype=dtype)
        with torch.no_grad():
            for p, o, n in zip(uniq, self.offsets, self.numels):
                view = slot_view(self.data, p, o)
                view.copy_(p.data)
                p.data = view
                if p.grad is not None:
                    g = slot_view(self.grad, p, o)
                    g.copy_(p.grad)
                    p.grad = g
                p._tdp_gslot = (self.grad, o)
                p._tdp_arena = self

    def index(self, p) -> int:
        for i, q in enumerate(self.params):
            if q is p:
                return i
        raise KeyError("parameter not in arena")

    def grad_view(self, i: int) -> torch.Tensor:
        return slot_view(self.grad, self.params[i], self.offsets[i])

    def is_arena_grad(self, i: int) -> bool:
        g = self.params[i].grad
        return g is not None and g.data_ptr() == self.grad.data_ptr() + \
            self.offsets[i] * self.grad.element_size()

    def new_state(self) -> torch.Tensor:
        """A zeroed buffer with the arena's layout (optimizer state: momentum, exp_avg, ...)."""
        return torch.zeros_like(self.data)

    def relayout(self, order):
        """Re-lay the arena out with the parameters in ``order`` (indices into ``self.params``):
        DDP's bucket rebuild from the observed gradient-ready order (torch
        ``Reducer::rebuild_buckets``, TORCH/nn/parallel/distributed.py:1199-1229). Parameter data
        and arena gradients move to fresh buffers; ``p.data`` / ``p.grad`` / grad slots follow.
        Returns ``remap(buf) -> new_buf`` that moves any other arena-shaped buffer (optimizer
        state) the same way. The arena object keeps its identity."""
        order = list(order)
        if sorted(order) != list(range(len(self.params))):
            raise ValueError("relayout order must be a permutation of the parameter indices")
        old_off = list(self.offsets)
        params = [self.params[i] for i in order]
        offsets, off = [], 0
        for p in params:
            offsets.append(off)
            off = _round_up(off + p.numel(), ALIGN)
        numel = max(off, ALIGN)
        moves = [(old_off[i], offsets[k], self.numels[i]) for k, i in enumerate(order)]

        def remap(buf: torch.Tensor) -> torch.Tensor:
            new = torch.zeros(numel, device=buf.device, dtype=buf.dtype)
            for src, dst, n in moves:
                new[dst: dst + n].copy_(buf[src: src + n])
            return new

        had_grad = [self.is_arena_grad(i) for i in range(len(self.params))]
        data, grad = remap(self.data), remap(self.grad)
        with torch.no_grad():
            for k, i in enumerate(order):
                p, o = self.params[i], offsets[k]
                p.data = slot_view(data, p, o)
                p._tdp_gslot = (grad, o)
                if had_grad[i]:
                    p.grad = slot_view(grad, p, o)
        self.params, self.offsets = params, offsets
        self.numels = [p.numel() for p in params]
        self.numel, self.data, self.grad = numel, data, grad
        return remap

    def state_view(self, buf: torch.Tensor, i: int) -> torch.Tensor:
        return slot_view(buf, self.params[i], self.offsets[i])


def arena_of(params):
    """The ParamArena holding exactly `params` (in any order), or None."""
    params = list(params)
    if not params:
        return None
    a = getattr(params[0], "_tdp_arena", None)
    if a is None or len(a.params) != len(params):
        return None
    ids = {id(p) for p in a.params}
    if any(id(p) not in ids or getattr(p, "_tdp_arena", None) is not a for p in params):
        return None
    if len({id(p) for p in params}) != len(params):
        return None
    return a


def flatten_module(module: torch.nn.Module, device=None) -> ParamArena:
    """Put every trainable fp32 parameter of `module` into one arena (backward order)."""
    existing = arena_of([p for p in module.parameters() if p.requires_grad])
    if existing is not None:
        return existing
    params = [p for p in module.parameters() if p.requires_grad]
    return ParamArena(list(reversed(params)), device=device)


class BufferArena:
    """A module's buffers packed into one flat tensor per (device, dtype), so DDP's per-forward
    buffer broadcast is one collective per dtype with no copies (ResNet-50:
    2 broadcasts -- float running stats, int64 num_batches_tracked -- instead of 160)."""

    def __init__(self, module: torch.nn.Module):
        groups = {}
        for b in module.buffers():
            groups.setdefault((b.device, b.dtype), []).append(b)
        self.flats = []
        for (dev, dt), bufs in groups.items():
            total, offs = 0, []
            for b in bufs:
                offs.append(total)
                total = _round_up(total + b.numel(), ALIGN)
            flat = torch.zeros(max(total, ALIGN), device=dev, dtype=dt)
            with torch.no_grad():
                for b, o in zip(bufs, offs):
                    v = flat[o: o + b.numel()].view(b.shape)
                    v.copy_(b)
                    b.data = v
            self.flats.append(flat)
