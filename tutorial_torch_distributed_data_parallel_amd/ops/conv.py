"""2-D convolution (+ fused bias / ReLU) on the native implicit-GEMM MFMA kernels.

Replaces MIOpen for the CNN models (§2.5 K1/K4/K6-K8 forward, K22 backward;
torchvision AlexNet features, REF/data_and_toy_model.py:41-45; ResNet-50 for the "ResNet-50-sized
CNN" config). Three kernels, none of which materialises an im2col buffer (``csrc/conv.hip``):
  * forward  ``y = relu?(conv(x, W) + b)`` -- bias and ReLU in the epilogue (K2 disappears);
  * input gradient (dgrad) -- strided convs handled by the divisibility test in the gather;
  * weight gradient (wgrad) -- split-K over the N*P*Q pixel reduction, written straight into the
    DDP gradient arena (``_grad.grad_dest``).
The ReLU mask and the per-channel bias gradient are one pass over ``dy`` (``chan_relu_bias_bwd``).
CPU tensors run ``torch.nn.functional.conv2d`` (the oracle of the CPU tests).
Groups and dilation are not supported (no model here uses them).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .._native import native
from ._grad import grad_dest, needs


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


class _Conv2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, stride, padding, relu: bool):
        C = native()
        sh, sw = stride
        ph, pw = padding
        y = C.conv2d_fwd(x, weight, bias, sh, sw, ph, pw, relu)
        ctx.geom = (sh, sw, ph, pw)
        ctx.relu = relu
        ctx.params = (weight, bias)
        ctx.x_shape = list(x.shape)
        ctx.save_for_backward(x, weight, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        C = native()
        x, weight, y = ctx.saved_tensors
        w_param, b_param = ctx.params
        sh, sw, ph, pw = ctx.geom
        dy = dy.contiguous()
        want_db = b_param is not None and needs(ctx, 2)
        db = grad_dest(b_param) if want_db else None
        # one pass: ReLU mask (g = dy * (y > 0)) and the per-channel bias gradient
        if ctx.relu or want_db:
            g = C.chan_relu_bias_bwd(dy, y if ctx.relu else None, db)
        else:
            g = dy
        dx = dw = None
        if needs(ctx, 1):
            dw = grad_dest(w_param)
            C.conv2d_wgrad(g, x, dw, sh, sw, ph, pw, 0.0)
        if needs(ctx, 0):
            dx = C.conv2d_dgrad(g, weight, ctx.x_shape, sh, sw, ph, pw)
        return dx, dw, db, None, None, None


def conv2d(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None,
           stride=1, padding=0, relu: bool = False) -> torch.Tensor:
    """``relu?(conv2d(x, weight, bias, stride, padding))`` for NCHW float32 tensors."""
    stride, padding = _pair(stride), _pair(padding)
    if not x.is_cuda:
        y = F.conv2d(x, weight, bias, stride, padding)
        return F.relu(y) if relu else y
    if x.dtype != torch.float32:
        raise TypeError(f"native conv2d expects float32 activations, got {x.dtype}")
    return _Conv2dFn.apply(x.contiguous(), weight.contiguous(), bias, stride, padding, relu)


def bias_relu_backward_reference(dy, y, bias_needed: bool):
    """CPU oracle of ``chan_relu_bias_bwd`` (used by tests)."""
    g = dy * (y > 0) if y is not None else dy
    db = g.sum(dim=(0, 2, 3)) if bias_needed else None
    return g, db
