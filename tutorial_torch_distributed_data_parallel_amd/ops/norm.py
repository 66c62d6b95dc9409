"""Batch norm / SyncBatchNorm autograd function over the native kernels (``csrc/norm.hip``).

Protocol (same as torch's SyncBatchNorm, TORCH/nn/modules/_functions.py:7-209):
  forward : local [mean | var | count]  --all_gather-->  count-weighted merge (+ running stats)
            --> normalise (optionally with a fused ReLU)
  backward: local [sum_dy | sum_dy_xmu] (+ local dW, dB straight into the grad arena)
            --all_reduce(sum)--> dx
With ``group=None`` the same kernels implement plain BatchNorm (one "rank").
On CPU the identical protocol runs on torch ops (``_TorchKernels``), which is what the gloo
multi-process tests exercise.

A batch of rows (BatchNorm1d, N <= 512 rows, C % 16 == 0) runs the whole-column kernels instead
(a workgroup owns 16 channels and every row): one launch per direction at one rank
(``bn1d_local_fwd`` / ``bn1d_local_bwd``, the latter also applying the fused optimizer to w / b),
``bn1d_moments`` -> all-gather -> ``bn1d_gathered_fwd`` and ``bn1d_sums`` -> all-reduce under
SyncBatchNorm (``set_local1d`` / ``set_sync1d`` switch back to the split kernels).

Reference: the README's SyncBatchNorm pitfall (/root/reference/README.md:79-81) -- BatchNorm
statistics must be synced across ranks, via ``convert_sync_batchnorm`` before wrapping in DDP.
"""
from __future__ import annotations


import torch
import torch.nn.functional as F

from .._native import native
from ._grad import bias_epilogue, grad_dest, hand_off, needs
from .linear import attach_planes, planes_input_fit


class _TorchKernels:
    """CPU reference of the five native batch-norm kernels (same tensor contracts)."""

    @staticmethod
    def _view(x):
        N, C = x.shape[0], x.shape[1]
        return x.reshape(N, C, -1)

    def bn_moments(self, x):
        v = self._view(x)
        C = v.shape[1]
        mean = v.mean(dim=(0, 2))
        var = v.var(dim=(0, 2), unbiased=False)
        cnt = torch.tensor([float(v.shape[0] * v.shape[2])], dtype=x.dtype)
        return [torch.cat([mean, var, cnt])[: 2 * C + 1]]

    def bn_merge(self, gathered, C, eps, momentum, rmean, rvar, num_batches=None):
        g = gathered.reshape(-1, 2 * C + 1)
        g = g[g[:, 2 * C] > 0]
        n = g[:, 2 * C: 2 * C + 1]
        total = n.sum()
        mean = (g[:, :C] * n).sum(0) / total
        m2 = (g[:, C: 2 * C] * n + n * (g[:, :C] - mean) ** 2).sum(0)
        var = m2 / total
        if num_batches is not None:
            num_batches.add_(1)
        if rmean is not None:
            unbiased = m2 / (total - 1) if total > 1 else var
            rmean.mul_(1 - momentum).add_(mean, alpha=momentum)
            rvar.mul_(1 - momentum).add_(unbiased, alpha=momentum)
        return torch.cat([mean, torch.rsqrt(var + eps), total.reshape(1)])

    def bn_elemt(self, x, stats, w, b, relu, residual=None):
        C = x.shape[1]
        shape = (1, C) + (1,) * (x.dim() - 2)
        y = (x - stats[:C].view(shape)) * stats[C: 2 * C].view(shape)
        if w is not None:
            y = y * w.view(shape)
        if b is not None:
            y = y + b.view(shape)
        if residual is not None:
            y = y + residual
        return F.relu(y) if relu else y

    def bn_bwd_reduce(self, dy, x, stats, y, dw, db, beta):
        C = x.shape[1]
        if y is not None:
            dy = dy * (y > 0)
        dv, xv = self._view(dy), self._view(x)
        s_dy = dv.sum(dim=(0, 2))
        s_dyx = (dv * (xv - stats[:C].view(1, C, 1))).sum(dim=(0, 2))
        if dw is not None:
            dw.copy_(s_dyx * stats[C: 2 * C])
        if db is not None:
            db.copy_(s_dy)
        return torch.cat([s_dy, s_dyx])

    def bn_bwd_elemt(self, dy, x, stats, w, sums, y, residual_grad=False):
        C = x.shape[1]
        shape = (1, C) + (1,) * (x.dim() - 2)
        if y is not None:
            dy = dy * (y > 0)
        cnt = stats[2 * C]
        inv = stats[C: 2 * C].view(shape)
        mdy = (sums[:C] / cnt).view(shape)
        mdyx = (sums[C:] / cnt).view(shape)
        dx = (dy - mdy - (x - stats[:C].view(shape)) * inv * inv * mdyx) * inv
        if w is not None:
            dx = dx * w.view(shape)
        return [dx, dy] if residual_grad else [dx]


_TORCH_K = _TorchKernels()




_LOCAL1D = True  # one-rank BatchNorm1d in one launch per direction (set_local1d: A/B, tests)
_LOCAL1D_UPDATE = True  # ... whose backward also applies the fused optimizer to w / b
_SYNC1D = True  # ... and SyncBatchNorm's local halves (set_sync1d: A/B, tests)


def set_sync1d(on: bool) -> bool:
    """Turn the whole-column SyncBatchNorm halves (moments; merge + normalisation; sums) on/off;
    returns the previous setting."""
    global _SYNC1D
    old, _SYNC1D = _SYNC1D, bool(on)
    return old


def set_local1d(on: bool, update: bool | None = None) -> bool:
    """Turn the one-launch one-rank BatchNorm1d path on/off (``update``: its in-place optimizer
    step on w / b); returns the previous setting of the path."""
    global _LOCAL1D, _LOCAL1D_UPDATE
    old, _LOCAL1D = _LOCAL1D, bool(on)
    if update is not None:
        _LOCAL1D_UPDATE = bool(update)
    return old


def _is_nhwc(x) -> bool:
    return x.dim() == 4 and not x.is_contiguous() and \
        x.is_contiguous(memory_format=torch.channels_last)


def _rows(x):
    return x.permute(0, 2, 3, 1).reshape(-1, x.shape[1])


def _unrows(y2, shape4):
    N, C, H, W = shape4
    return y2.view(N, H, W, C).permute(0, 3, 1, 2)


def _kernels(x):
    return native() if x.is_cuda else _TORCH_K


class _BatchNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, relu, group,
                residual, num_batches, sink=None, part=None):
        K = _kernels(x)
        C = x.shape[1]
        # channels_last (NHWC) activations are a [pixels, C] matrix: the BatchNorm1d kernels
        # (64 adjacent channels per workgroup, coalesced) apply unchanged
        ctx.nhwc = x.is_cuda and _is_nhwc(x)
        ctx.shape4 = tuple(x.shape)
        x = _rows(x) if ctx.nhwc else x.contiguous()
        if residual is not None:
            residual = _rows(residual.contiguous(memory_format=torch.channels_last)) \
                if ctx.nhwc else residual.contiguous()
        # [rows, C % 4] form on the GPU: the backward reads a 1-byte-per-4-channels ReLU mask
        # instead of the float output (1/16 of the bytes, twice per backward)
        mask = None
        rows4 = x.is_cuda and x.dim() == 2 and C % 4 == 0
        if relu and rows4:
            mask = torch.empty((x.shape[0], C // 4), dtype=torch.uint8, device=x.device)
        # a BatchNorm1d output feeding a skinny Linear: its bf16 split planes from the same pass
        pl = None
        if rows4 and not ctx.nhwc and planes_input_fit(x.shape[0], C):
            pl = torch.empty((3, x.shape[0], C), dtype=torch.bfloat16, device=x.device)
        y = None
        # one rank, a batch of rows (BatchNorm1d): statistics + normalisation in one launch, and
        # the backward likewise (csrc/norm.hip bn1d_local_fwd / bn1d_local_bwd)
        ctx.local1d = False
        if group is None and rows4 and not ctx.nhwc and residual is None and part is None and \
                _LOCAL1D:
            r = native().bn1d_local_fwd(x, weight, bias, relu, float(eps), float(momentum),
                                        rmean=running_mean, rvar=running_var,
                                        num_batches=num_batches, mask_out=mask, planes_out=pl)
            if r:
                y, stats = r
                ctx.local1d = True
        # SyncBatchNorm over a batch of rows: the same whole-column kernels around the gather
        # (moments in one launch; merge + normalisation in one launch)
        sync1d = group is not None and rows4 and not ctx.nhwc and residual is None and \
            part is None and _LOCAL1D and _SYNC1D
        st = None
        if y is None and sync1d:
            st = native().bn1d_moments(x)
            if st is not None and st.numel() == 0:
                st = None
            if st is not None:
                gathered = group.all_gather_flat(st)
                r = native().bn1d_gathered_fwd(x, gathered, weight, bias, relu, float(eps),
                                               float(momentum), rmean=running_mean,
                                               rvar=running_var, num_batches=num_batches,
                                               mask_out=mask, planes_out=pl)
                if r:
                    y, stats = r
                    ctx.local1d = True
                else:  # (unaligned parameters) the split merge + normalisation, same moments
                    stats = K.bn_merge(gathered, C, eps, momentum, running_mean, running_var,
                                       num_batches)
                    kw = {} if mask is None else {"mask_out": mask}
                    if pl is not None:
                        kw["planes_out"] = pl
                    y = K.bn_elemt(x, stats, weight, bias, relu, residual, **kw)
        if y is None:
            if part is not None and ctx.nhwc:
                # statistics from the producing convolution's GEMM epilogue (per-tile Chan merge)
                st = native().bn_moments_partials(part, float(x.shape[0]))
            else:
                st = K.bn_moments(x)[0]
        if y is None and group is None and rows4:
            # one rank: bn_merge's work runs inside the normalisation pass (one launch fewer)
            r = native().bn_elemt_local(x, st, weight, bias, relu, float(eps), float(momentum),
                                        rmean=running_mean, rvar=running_var,
                                        num_batches=num_batches, mask_out=mask, planes_out=pl,
                                        residual=residual)
            if r:
                y, stats = r
        if y is None:
            gathered = group.all_gather_flat(st) if group is not None else st
            stats = K.bn_merge(gathered, C, eps, momentum, running_mean, running_var,
                               num_batches)
            kw = {} if mask is None else {"mask_out": mask}
            if pl is not None:
                kw["planes_out"] = pl
            y = K.bn_elemt(x, stats, weight, bias, relu, residual, **kw)
        if pl is not None:
            attach_planes(y, pl)
        ctx.params = (weight, bias)
        ctx.relu = relu
        ctx.group = group
        ctx.has_res = residual is not None
        ctx.sink = sink
        ctx.save_for_backward(x, weight, stats, y if (relu and mask is None) else None, mask)
        return _unrows(y, ctx.shape4) if ctx.nhwc else y

    @staticmethod
    def backward(ctx, dy):
        x, weight, stats, y, mask = ctx.saved_tensors
        K = _kernels(x)
        dy = _rows(dy.contiguous(memory_format=torch.channels_last)) if ctx.nhwc \
            else dy.contiguous()
        w_param, b_param = ctx.params
        dw = grad_dest(w_param) if (w_param is not None and needs(ctx, 1)) else None
        db = grad_dest(b_param) if (b_param is not None and needs(ctx, 2)) else None
        mk = {} if mask is None else {"mask": mask}
        if ctx.local1d and ctx.group is None:
            # one launch: the column sums, dw / db and dx (+ its planes) of a whole-rows batch
            pl = None
            if needs(ctx, 0) and planes_input_fit(x.shape[0], x.shape[1]):
                pl = torch.empty((3,) + tuple(x.shape), dtype=torch.bfloat16, device=x.device)
            # world size 1 + fused optimizer: the kernel that completes dw / db also applies the
            # update to w / b (hand_off: their slots go to autograd unwritten)
            kw = {}
            be_w = bias_epilogue(w_param) if (dw is not None and _LOCAL1D_UPDATE) else None
            be_b = bias_epilogue(b_param) if (db is not None and _LOCAL1D_UPDATE) else None
            # only a DDP reducer backend (a tensor-sharded wrapper's target has no span)
            be_w = be_w if (be_w is not None and be_w[2] is not None) else None
            be_b = be_b if (be_b is not None and be_b[2] is not None) else None
            if be_w is not None and (be_b is None or be_b[0] is be_w[0]):
                kw.update(backend=be_w[0], w_offset=be_w[1], w_span=be_w[2])
            else:
                be_w = None
            if be_b is not None and (not kw or kw["backend"] is be_b[0]):
                kw.update(backend=be_b[0], b_offset=be_b[1], b_span=be_b[2])
            else:
                be_b = None
            dx = native().bn1d_local_bwd(dy, x, stats, weight, mask=mask, dw=dw, db=db,
                                         planes_out=pl, **kw)
            if be_w is not None:
                hand_off(w_param, dw)
            if be_b is not None:
                hand_off(b_param, db)
            if pl is not None:
                attach_planes(dx, pl)
            return (dx if needs(ctx, 0) else None), dw, db, None, None, None, None, None, None, \
                None, None, None, None
        sums = None
        if ctx.local1d:
            # SyncBatchNorm (ctx.group set): the local sums + dw / db in one launch
            sums = native().bn1d_sums(dy, x, stats, mask=mask, dw=dw, db=db)
            if sums is not None and sums.numel() == 0:
                sums = None
        if sums is None:
            sums = K.bn_bwd_reduce(dy, x, stats, y, dw, db, 0.0, **mk)
        dx = dres = None
        want_res = ctx.has_res and needs(ctx, 9)
        if needs(ctx, 0) or want_res:
            if ctx.group is not None:
                ctx.group.all_reduce_sum_(sums)
            # one pass: dx, and the residual input's gradient (the ReLU-masked dy) when fused;
            # a BatchNorm1d input gradient feeding a skinny Linear's backward also leaves as planes
            pl = None
            if needs(ctx, 0) and x.is_cuda and not ctx.nhwc and x.dim() == 2 and \
                    x.shape[1] % 4 == 0 and planes_input_fit(x.shape[0], x.shape[1]):
                pl = torch.empty((3,) + tuple(x.shape), dtype=torch.bfloat16, device=x.device)
                mk = dict(mk, planes_out=pl)
            out = K.bn_bwd_elemt(dy, x, stats, weight, sums, y, want_res, **mk)
            if pl is not None:
                attach_planes(out[0], pl)
            dx = out[0] if needs(ctx, 0) else None
            dres = out[1] if want_res else None
            if ctx.nhwc:
                dx = _unrows(dx, ctx.shape4) if dx is not None else None
                dres = _unrows(dres, ctx.shape4) if dres is not None else None
            if dres is not None and ctx.sink is not None:
                dres = ctx.sink.deposit(dres)  # the forked block input's shared gradient
        return dx, dw, db, None, None, None, None, None, None, dres, None, None, None


def _conv_stats(x):
    """Per-tile statistics a producing convolution attached to ``x`` (ops/conv.py
    ``bn_stats``), if they still describe it (same version: not modified in place since)."""
    tag = getattr(x, "_tdp_bn_part", None)
    if tag is None or tag[1] != x._version or tag[0].shape[2] != x.shape[1]:
        return None
    return tag[0]


def batch_norm(x: torch.Tensor, running_mean: torch.Tensor | None,
               running_var: torch.Tensor | None, weight: torch.Tensor | None = None,
               bias: torch.Tensor | None = None, training: bool = True, momentum: float = 0.1,
               eps: float = 1e-5, relu: bool = False, group=None, residual=None,
               num_batches_tracked=None, residual_grad_into=None) -> torch.Tensor:
    """``relu?(batch_norm(x) [+ residual])`` over dim 1 of x ([N, C] or [N, C, *]); ``group``
    makes it synchronous; ``num_batches_tracked`` (training) is incremented on the device;
    ``residual_grad_into`` (a ``SharedGrad``) receives the residual's gradient."""
    if training:
        if residual is not None and x.is_cuda and not (x.shape[1] % 4 == 0 and (
                x.dim() == 2 or _is_nhwc(x))):
            # the fused residual exists in the [rows, C % 4 == 0] kernels only
            y = _BatchNormFn.apply(x, weight, bias, running_mean, running_var, float(momentum),
                                   float(eps), False, group, None, num_batches_tracked)
            y = y + residual
            return F.relu(y) if relu else y
        return _BatchNormFn.apply(x, weight, bias, running_mean, running_var, float(momentum),
                                  float(eps), bool(relu), group, residual, num_batches_tracked,
                                  residual_grad_into, _conv_stats(x))
    if residual is not None:
        y = batch_norm(x, running_mean, running_var, weight, bias, False, momentum, eps, False)
        y = y + residual
        return F.relu(y) if relu else y
    if x.is_cuda and not (torch.is_grad_enabled() and (x.requires_grad or (
            weight is not None and weight.requires_grad))):
        if _is_nhwc(x):
            y2 = native().bn_eval(_rows(x), running_mean, running_var, weight, bias, float(eps),
                                  bool(relu))
            return _unrows(y2, tuple(x.shape))
        return native().bn_eval(x.contiguous(), running_mean, running_var, weight, bias,
                                float(eps), bool(relu))
    # inference-mode BN that must be differentiated (frozen-BN fine-tuning): a per-channel affine
    # map y = x * scale + shift, differentiated by autograd through plain elementwise ops
    shape = (1, x.shape[1]) + (1,) * (x.dim() - 2)
    scale = torch.rsqrt(running_var + eps)
    if weight is not None:
        scale = scale * weight
    shift = -running_mean * scale
    if bias is not None:
        shift = shift + bias
    y = x * scale.view(shape) + shift.view(shape)
    return F.relu(y) if relu else y
