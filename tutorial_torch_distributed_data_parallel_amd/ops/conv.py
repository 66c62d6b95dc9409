"""2-D convolution (+ fused bias / ReLU) on the native implicit-GEMM MFMA kernels.

Replaces MIOpen for the CNN models (§2.5 K1/K4/K6-K8 forward, K22 backward;
torchvision AlexNet features, REF/data_and_toy_model.py:41-45; ResNet-50 for the "ResNet-50-sized
CNN" config). No im2col buffer is ever materialised.

Main path -- channels_last (NHWC) activations on the LDS-DMA MFMA GEMM pipeline
(``csrc/gemm_f32_fast.hip``, implicit operand sources):
  * forward  ``y[(n,p,q)][co] = relu?(sum_(r,s,c) x[n][p*sh-ph+r][q*sw-pw+s][c] * W[co][c][r][s] + b)``
    -- K is ordered (r, s, c) so every 16-B DMA chunk is 4 contiguous channels of one pixel;
  * input gradient -- the same gather on ``dy`` with the transpose-stride test;
  * weight gradient -- ``dy^T`` (a plain [pixels][Cout] matrix) times shifted-pixel rows of ``x``,
    split-K over the N*P*Q reduction.
  Outputs are channels_last, so a 1x1 convolution IS a GEMM ([N*H*W, C] x [C, Cout]); batch norm
  and the ReLU/bias backward treat NHWC tensors as [pixels, C] matrices. Weights are
  channels_last parameters (logical [Cout, C, R, S]: state_dict / checkpoints unchanged) whose
  [Cout][R][S][C] memory every kernel reads or writes directly (see _ConvNHWCFn).
  Input channels that are not a multiple of 4 (the RGB stem) are zero-padded to 4, natively.
Fallback -- NCHW register-staged implicit GEMM (``csrc/conv.hip``) for shapes the NHWC path does
not take (channel counts not a multiple of 4 beyond the stem, non power-of-two strides in dgrad).
CPU tensors run ``torch.nn.functional.conv2d`` (the oracle of the CPU tests).
Groups and dilation are not supported (no model here uses them).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .._native import native
from . import plan_db
from ._grad import SharedGrad, grad_dest, needs


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


class _Conv2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, stride, padding, relu: bool, sink=None):
        C = native()
        sh, sw = stride
        ph, pw = padding
        y = C.conv2d_fwd(x, weight, bias, sh, sw, ph, pw, relu)
        ctx.sink = sink
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
            if ctx.sink is not None:
                dx = ctx.sink.deposit(dx)
        return dx, dw, db, None, None, None, None


_CL = torch.channels_last


def _rows(t):
    """[N, C, H, W] channels_last tensor -> its [N*H*W, C] storage as a 2-D view."""
    return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1])


def _as_cl(C, t, channels: int | None = None):
    """``t`` as a channels_last tensor with ``channels`` channels (zero-padded): ``t`` itself
    when it already is one, else ONE native strided copy (csrc/elementwise.hip copy4d)."""
    n, c, h, w = t.shape
    channels = c if channels is None else channels
    if channels == c and t.is_contiguous(memory_format=_CL):
        return t
    base = getattr(t, "_tdp_padded_base", None)
    if base is not None and tuple(base.shape) == (n, h, w, channels) and \
            t.data_ptr() == base.data_ptr() and t.stride() == (h * w * channels, 1, w * channels,
                                                                 channels):
        # a channel-padded channels_last batch (data/synthetic.py): its zero-filled storage IS
        # the padded NHWC operand
        return base.permute(0, 3, 1, 2)
    out = torch.empty((n, channels, h, w), device=t.device, dtype=t.dtype, memory_format=_CL)
    C.copy4d(out, t)
    return out


class _ConvNHWCFn(torch.autograd.Function):
    """Weights are channels_last parameters ([Cout][R][S][C] memory, nn/modules.py Conv2d): the
    forward reads them as the GEMM's K-contiguous B, the input gradient gathers its taps straight
    from them (csrc/gemm_f32_fast.hip WTap), and the weight gradient is written straight into
    the parameter's gradient slot in that layout -- no per-step permute / pad / copy-back. Only
    the RGB stem (3 channels, padded to 4 for the 16-B DMA chunks) repacks, natively."""

    @staticmethod
    def forward(ctx, x, weight, bias, stride, padding, relu: bool, sink=None, stats_box=None):
        C = native()
        N, Cin, H, W = x.shape
        Cout, _, R, S = weight.shape
        Cp = (Cin + 3) // 4 * 4
        sh, sw = stride
        ph, pw = padding
        xp = _as_cl(C, x, Cp)
        wt = _as_cl(C, weight, Cp)  # the parameter itself for every conv but the stem
        if stats_box is not None and bias is None and not relu:
            # the GEMM epilogue also emits the output's per-tile BN statistics (or None)
            y, st = C.conv_nhwc_fwd_stats(xp, wt.permute(0, 2, 3, 1), R, S, sh, sw, ph, pw)
            stats_box.append(st)
        else:
            y = C.conv_nhwc_fwd(xp, wt.permute(0, 2, 3, 1), bias, R, S, sh, sw, ph, pw, relu)
        ctx.geom = (R, S, sh, sw, ph, pw, Cin, Cp)
        ctx.sink = sink
        ctx.relu = relu
        ctx.params = (weight, bias)
        ctx.save_for_backward(xp, wt, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        C = native()
        xp, wt, y = ctx.saved_tensors
        w_param, b_param = ctx.params
        R, S, sh, sw, ph, pw, Cin, Cp = ctx.geom
        Cout = wt.shape[0]
        dy = _as_cl(C, dy)
        want_db = b_param is not None and needs(ctx, 2)
        db = grad_dest(b_param) if want_db else None
        # ReLU mask + bias gradient: one pass over dy viewed as [pixels, Cout]
        if ctx.relu or want_db:
            g2 = C.relu_bias_bwd(_rows(dy), _rows(y) if ctx.relu else None, db)
            g = g2.view(dy.shape[0], dy.shape[2], dy.shape[3], Cout).permute(0, 3, 1, 2)
        else:
            g = dy
        dx = dw = None
        if needs(ctx, 1):
            dw = grad_dest(w_param)
            if C.conv_wgrad_transposed(Cout, R, S, Cp):
                # dW^T [(r,s,c)][co] when it pads the 128-row MFMA tiles less (small Cout, Cout=192)
                dwT = torch.empty((R, S, Cp, Cout), device=dy.device, dtype=dy.dtype)
                C.conv_nhwc_wgrad(g, xp, dwT, R, S, sh, sw, ph, pw, 0.0)
                C.copy4d(dw, dwT.permute(3, 2, 0, 1))
            elif Cp == Cin and dw.permute(0, 2, 3, 1).is_contiguous():
                # straight into the gradient slot ([Cout][R][S][C] = the parameter's layout)
                C.conv_nhwc_wgrad(g, xp, dw.permute(0, 2, 3, 1), R, S, sh, sw, ph, pw, 0.0)
            else:
                dwt = torch.empty((Cout, R, S, Cp), device=dy.device, dtype=dy.dtype)
                C.conv_nhwc_wgrad(g, xp, dwt, R, S, sh, sw, ph, pw, 0.0)
                C.copy4d(dw, dwt.permute(0, 3, 1, 2))
        if needs(ctx, 0):
            sink = ctx.sink
            acc = sink.buf if (sink is not None and Cp == Cin) else None
            if sh == 1 and sw == 1:
                # with a shared residual-input gradient: accumulated by the GEMM (beta = 1)
                dx = C.conv_nhwc_dgrad_w(g, wt, list(xp.shape), sh, sw, ph, pw, out=acc,
                                         beta=0.0 if acc is None else 1.0)
            else:
                dx = _dgrad_phases(C, g, wt, xp.shape, R, S, sh, sw, ph, pw, into=acc)
            if Cp != Cin:
                dx = dx[:, :Cin]
            if sink is not None:
                dx = dx if acc is not None else sink.deposit(dx)
        return dx, dw, db, None, None, None, None, None


def _dgrad_phases(C, g, wt, x_shape, R, S, sh, sw, ph, pw, into=None):
    """Strided input gradient as sh*sw stride-1 GEMMs, one per output phase.

    dx pixels h = a + sh*i only receive taps r = r0 + sh*t with r0 = (a + ph) mod sh, from dy row
    p = i + da - t (da = (a + ph - r0) / sh): a stride-1 convolution over the phase sub-grid with
    the phase's taps, which the kernel gathers from the weight itself. This skips the
    (sh*sw - 1)/(sh*sw) of multiply-adds a direct gather spends on the zeros between strided
    taps (measured 4x on ResNet's stride-2 layers). ``into``: accumulate into that tensor
    instead (phases without taps leave it alone)."""
    N, Cp, H, W = x_shape
    acc = into is not None
    dx = into if acc else torch.empty(x_shape, device=g.device, dtype=g.dtype, memory_format=_CL)
    none = torch.empty((0, 0, 0, 0), device=g.device, dtype=g.dtype)
    for a in range(sh):
        r0 = (a + ph) % sh
        Rp, Hp, da = len(range(r0, R, sh)), len(range(a, H, sh)), (a + ph - r0) // sh
        for b in range(sw):
            s0 = (b + pw) % sw
            Sp, Wp, db = len(range(s0, S, sw)), len(range(b, W, sw)), (b + pw - s0) // sw
            if Hp == 0 or Wp == 0:
                continue
            view = dx[:, :, a::sh, b::sw]
            if Rp == 0 or Sp == 0:
                if not acc:
                    C.copy4d(view, none)  # no tap reaches this phase: zeros
                continue
            C.copy4d(view, C.conv_nhwc_dgrad_phase_w(g, wt, Hp, Wp, Rp, Sp, da, db, r0, s0, sh,
                                                     sw), accumulate=acc)
    return dx


FORCE_NCHW = False  # tests: route every conv through the NCHW fallback kernels


def _nhwc_ok(x, weight, stride):
    if FORCE_NCHW:
        return False
    Cin, Cout = weight.shape[1], weight.shape[0]
    pow2 = all(s > 0 and (s & (s - 1)) == 0 for s in stride)
    return (Cin % 4 == 0 or Cin < 4) and Cout % 4 == 0 and (pow2 or not x.requires_grad)


def conv2d(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None,
           stride=1, padding=0, relu: bool = False,
           grad_into: SharedGrad | None = None, bn_stats: bool = False) -> torch.Tensor:
    """``relu?(conv2d(x, weight, bias, stride, padding))`` for float32 [N, C, H, W] tensors.

    On the GPU the result is channels_last (NHWC memory, logical NCHW shape, as torch does for
    channels_last inputs). ``grad_into``: the input gradient goes into that shared buffer (a
    forked residual input, ops/_grad.py ``fork``). ``bn_stats``: the output will be
    batch-normalised -- the GEMM epilogue also computes its per-channel statistics, attached
    to the result for ``batch_norm`` (no moments pass over the output)."""
    stride, padding = _pair(stride), _pair(padding)
    if not x.is_cuda:
        y = F.conv2d(x, weight, bias, stride, padding)
        return F.relu(y) if relu else y
    if x.dtype != torch.float32:
        raise TypeError(f"native conv2d expects float32 activations, got {x.dtype}")
    if _nhwc_ok(x, weight, stride):
        plan_db.ensure_loaded(native())  # measured per-geometry plans (ops/plan_db.py)
        box = [] if bn_stats else None
        y = _ConvNHWCFn.apply(x, weight, bias, stride, padding, relu, grad_into, box)
        if box and box[0] is not None:
            y._tdp_bn_part = (box[0], y._version)  # ops/norm.py batch_norm consumes it
        return y
    return _Conv2dFn.apply(x.contiguous(), weight.contiguous(), bias, stride, padding, relu,
                           grad_into)


def bias_relu_backward_reference(dy, y, bias_needed: bool):
    """CPU oracle of ``chan_relu_bias_bwd`` (used by tests)."""
    g = dy * (y > 0) if y is not None else dy
    db = g.sum(dim=(0, 2, 3)) if bias_needed else None
    return g, db
