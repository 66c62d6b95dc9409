"""Pooling, dropout and residual add+ReLU over the native kernels (``csrc/pool.hip``).

SURVEY.md §2.5: K3/K5/K9 ``max_pool2d_with_indices`` and K20 its backward (a deterministic gather,
no atomics), K10/K21 ``adaptive_avg_pool2d`` (identity when the input already has the output size,
as for 224x224 AlexNet where the features end at 6x6), K11/K19 dropout (mask regenerated from a
counter-based hash in the backward instead of being stored) and the residual add+ReLU of ResNet
bottlenecks. CPU tensors run the ``torch.nn.functional`` reference.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .._native import native


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


_CL = torch.channels_last


def is_nhwc(x) -> bool:
    """channels_last memory that is not also plain-contiguous (1x1 spatial maps are both)."""
    return x.dim() == 4 and not x.is_contiguous() and x.is_contiguous(memory_format=_CL)


def _fmt(x):
    return _CL if is_nhwc(x) else torch.contiguous_format


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        ctx.nhwc = is_nhwc(x)
        if ctx.nhwc:
            y, idx = native().maxpool_nhwc_fwd(x, k, s, p)
        else:
            y, idx = native().maxpool2d_fwd(x, k, s, p)
        ctx.save_for_backward(idx)
        ctx.cfg = (list(x.shape), k, s, p)
        ctx.mark_non_differentiable(idx)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        shape, k, s, p = ctx.cfg
        if ctx.nhwc:
            dx = native().maxpool_nhwc_bwd(dy.contiguous(memory_format=_CL), idx, shape, k, s, p)
        else:
            dx = native().maxpool2d_bwd(dy.contiguous(), idx, shape, k, s, p)
        return dx, None, None, None


def max_pool2d(x, kernel_size, stride=None, padding=0):
    """Square-window max pooling (``ceil_mode=False``, no dilation)."""
    k = _pair(kernel_size)
    s = _pair(stride if stride is not None else kernel_size)
    p = _pair(padding)
    if not x.is_cuda:
        return F.max_pool2d(x, k, s, p)
    if k[0] != k[1] or s[0] != s[1] or p[0] != p[1]:
        raise NotImplementedError("native max_pool2d supports square windows only")
    return _MaxPoolFn.apply(x.contiguous(memory_format=_fmt(x)), k[0], s[0], p[0])


class _AvgPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, P, Q):
        ctx.shape = list(x.shape)
        ctx.nhwc = is_nhwc(x)
        if ctx.nhwc:
            return native().avgpool_nhwc_fwd(x, P, Q)
        return native().avgpool_fwd(x, P, Q)

    @staticmethod
    def backward(ctx, dy):
        if ctx.nhwc:
            return native().avgpool_nhwc_bwd(dy, ctx.shape), None, None
        return native().avgpool_bwd(dy, ctx.shape), None, None


def adaptive_avg_pool2d(x, output_size):
    P, Q = _pair(output_size)
    if x.shape[-2] == P and x.shape[-1] == Q:
        return x  # identity (torch launches a copy kernel here)
    if not x.is_cuda:
        return F.adaptive_avg_pool2d(x, (P, Q))
    return _AvgPoolFn.apply(x.contiguous(memory_format=_fmt(x)), P, Q)


class _FlattenNCHWFn(torch.autograd.Function):
    """channels_last [N, C, H, W] -> [N, C*H*W] in torch's (C, H, W) feature order (what the
    classifier weights expect, e.g. torchvision AlexNet's fc6), and back in the backward: one
    native strided copy each way (csrc/elementwise.hip copy4d) instead of ATen's direct_copy."""

    @staticmethod
    def forward(ctx, x):
        N, C, H, W = x.shape
        out = torch.empty((N, C, H, W), device=x.device, dtype=x.dtype)
        native().copy4d(out, x)
        ctx.shape = (N, C, H, W)
        return out.view(N, C * H * W)

    @staticmethod
    def backward(ctx, dy):
        N, C, H, W = ctx.shape
        gx = torch.empty((N, C, H, W), device=dy.device, dtype=dy.dtype,
                         memory_format=torch.channels_last)
        native().copy4d(gx, dy.contiguous().view(N, C, H, W))
        return gx


def flatten(x: torch.Tensor) -> torch.Tensor:
    """``torch.flatten(x, 1)`` with torch's feature order; a channels_last GPU activation is
    reordered natively (no ATen copy kernel)."""
    if x.is_cuda and x.dim() == 4 and x.dtype == torch.float32 and not x.is_contiguous() and \
            x.is_contiguous(memory_format=torch.channels_last):
        return _FlattenNCHWFn.apply(x)
    return x.reshape(x.shape[0], -1)


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, seed):
        ctx.cfg = (p, seed, _fmt(x))
        return native().dropout(x, p, seed)

    @staticmethod
    def backward(ctx, dy):
        p, seed, fmt = ctx.cfg
        # same (seed, memory index) hash -> same mask, same 1/(1-p) scale
        return native().dropout(dy.contiguous(memory_format=fmt), p, seed), None, None


def dropout(x, p: float = 0.5, training: bool = True, generator=None):
    """Inverted dropout. The per-call seed comes from torch's CPU generator (reproducible under
    ``torch.manual_seed``); inside a captured hipGraph the seed is fixed at capture."""
    if not training or p == 0.0:
        return x
    if p >= 1.0:
        return x * 0.0
    if not x.is_cuda:
        return F.dropout(x, p, True)
    seed = int(torch.randint(0, 2 ** 62, (1,), generator=generator).item())
    return _DropoutFn.apply(x.contiguous(memory_format=_fmt(x)), float(p), seed)


class _AddReluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        y = native().add_relu(a, b, True)
        ctx.fmt = _fmt(a)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        g = native().relu_mask(dy.contiguous(memory_format=ctx.fmt), y)
        return g, g


def add_relu(a, b):
    """``relu(a + b)`` -- the residual join of a ResNet block."""
    if not a.is_cuda:
        return F.relu(a + b)
    fmt = _fmt(a)
    return _AddReluFn.apply(a.contiguous(memory_format=fmt), b.contiguous(memory_format=fmt))
