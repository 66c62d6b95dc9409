"""Linear (+ fused ReLU) on the native fp32 MFMA GEMM.

Forward, input-gradient and weight-gradient are each ONE kernel (plus a split-K combine when the
tile grid alone cannot fill 256 CUs):
  * forward  ``y = relu(x W^T + b)``: bias and ReLU in the GEMM epilogue;
  * backward: one pass applies the ReLU mask ``y > 0`` to ``dy`` (K18, ``relu_bias_bwd``); the
    weight-gradient GEMM also reduces the bias gradient from its staged A tiles (K17), both
    GEMMs read the masked gradient through their LDS-DMA pipelines, and the weight gradient lands
    directly in the DDP gradient arena (K23, see ``_grad.py``).
On CPU the same math runs through ``torch.nn.functional`` (the reference implementation used by
the gloo/CPU tests). Reference behaviour: torchvision AlexNet's classifier Linear/ReLU layers
(REF/data_and_toy_model.py:41-45).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


from .._native import native
from ._grad import (bias_epilogue, epilogue_target, factor_target, grad_dest, hand_off, needs,
                    note_use)

# Skinny GEMMs (batch rows against thousands of features) read their activation operand from
# its exact bf16 split planes (csrc/gemm_planes.hip): split once by the producer instead of once
# per column tile inside the GEMM (set_planes(False) keeps the in-kernel split: A/B measurements).
_PLANES = True


# Rows up to which the activation operand goes pre-split: a batch per rank (M = 128), or the
# node's batch of the tensor-sharded step (M = W * 128 <= 1024: profiles/r9/tp_planes_r9.md)
PLANES_MAX_ROWS = 1024


def planes_fit(M: int, N: int, K: int) -> bool:
    """The planes GEMM applies: few rows (a batch), K a multiple of its 32-deep tile, wide N."""
    return _PLANES and M <= PLANES_MAX_ROWS and K % 32 == 0 and K >= 256 and N % 4 == 0 and \
        N >= 512


def planes_input_fit(M: int, K: int) -> bool:
    """A [M, K] activation may feed a planes GEMM (its producer should emit the planes)."""
    return _PLANES and M <= PLANES_MAX_ROWS and K % 32 == 0 and K >= 256


def _al16(*ts) -> bool:
    """Every given tensor (None skipped) has 16-B aligned rows (the planes GEMM's 16-B loads)."""
    return all(t is None or (t.data_ptr() % 16 == 0 and (t.dim() < 2 or t.stride(0) % 4 == 0))
               for t in ts)


_EARLY_PREV_G = True  # the consumer's backward starts the previous layer's g gather


def set_early_prev_g(on: bool) -> bool:
    """Turn the one-layer-early g gather on/off (A/B: scripts/run_with_variant.py); returns the
    previous setting."""
    global _EARLY_PREV_G
    old, _EARLY_PREV_G = _EARLY_PREV_G, bool(on)
    return old


_PAIR_WGRAD = True  # world size 1: consecutive weight-gradient + optimizer GEMMs share a launch


def set_pair_wgrad(on: bool) -> bool:
    """Turn the paired weight-gradient + optimizer launch on/off (A/B, tests); returns the
    previous setting."""
    global _PAIR_WGRAD
    old, _PAIR_WGRAD = _PAIR_WGRAD, bool(on)
    return old


def set_planes(on: bool) -> bool:
    """Turn the planes path on/off (tests, A/B); returns the previous setting."""
    global _PLANES
    old, _PLANES = _PLANES, bool(on)
    return old


def attach_planes(t: torch.Tensor, planes: torch.Tensor) -> None:
    """Record that ``planes`` are the bf16 split of ``t``'s current contents."""
    t._tdp_planes = (planes, t._version, t.data_ptr(), tuple(t.shape))


def has_planes(t: torch.Tensor) -> bool:
    """``t`` carries its producer's split planes (planes_of would not split it)."""
    for src in (t, t._base):
        rec = getattr(src, "_tdp_planes", None) if src is not None else None
        if rec is not None and rec[1] == src._version and rec[2] == t.data_ptr():
            return True
    return False


def planes_of(t: torch.Tensor) -> torch.Tensor:
    """The split planes of a 2-D fp32 tensor: the producer's (attach_planes) when they still
    describe it, else one split_planes pass."""
    for src in (t, t._base):  # a reshape view of the producer's tensor shares its planes
        rec = getattr(src, "_tdp_planes", None) if src is not None else None
        if rec is not None and rec[1] == src._version and rec[2] == t.data_ptr() and \
                rec[0][0].numel() == t.numel() and rec[0].shape[1] == t.shape[0] and \
                t.is_contiguous():
            return rec[0] if rec[0].shape[1:] == t.shape else rec[0].view(3, *t.shape)
    if t.stride(-1) != 1 or t.stride(0) % 4 or t.data_ptr() % 16:
        t = t.contiguous()
    return native().split_planes(t)


def _pregated(dy: torch.Tensor, y: torch.Tensor) -> bool:
    """``dy`` was already multiplied by (y > 0) by the consumer that produced it (its
    input-gradient epilogue gated by this layer's ReLU output, see _LinearFn.backward)."""
    return getattr(dy, "_tdp_gated_by", None) == (y.data_ptr(), tuple(y.shape)) and \
        dy.shape == y.shape and dy.stride() == y.stride()


def _mark_gated(dx: torch.Tensor, gate: torch.Tensor) -> None:
    dx._tdp_gated_by = (gate.data_ptr(), tuple(gate.shape))


def _prefetch_prev_g(ctx, dx: torch.Tensor):
    """The gated dx of a layer whose input is a fused Linear+ReLU output IS that previous
    layer's output gradient g: a factored previous weight starts its g gather now, right after
    the GEMM that produced dx, so on the comm stream it precedes this layer's own collectives
    (parameter all-gather, bucket all-reduce) instead of queueing behind them
    (DDP.factor_prefetch_g; docs/COMM_MODEL.md "early g gather"). Returns the DDP that issued
    it (the caller flushes its fork after the GEMM's node), else None."""
    if ctx.prev_w is None or not _EARLY_PREV_G or not dx.is_cuda:
        return None
    prev = factor_target(ctx.prev_w)
    return prev if prev is not None and prev.factor_prefetch_g(ctx.prev_w, dx) else None


def _dx_buffer(ctx, x2: torch.Tensor) -> torch.Tensor:
    """The input gradient of a layer whose input is the ReLU output of a factored Linear IS that
    layer's g (this layer's epilogue applies the mask): written straight into the factored job's
    gather slot (DDP.factor_g_dest), the g all-gather then runs in place; else a fresh tensor."""
    if ctx.prev_w is not None and ctx.gate_in and x2.is_cuda:
        prev = factor_target(ctx.prev_w)
        if prev is not None:
            d = prev.factor_g_dest(ctx.prev_w, x2.shape[0])
            if d is not None and d.shape == x2.shape:
                return d
    return torch.empty_like(x2)


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x2, weight, bias, relu: bool, gate_in: bool, fac=None, prev=None):
        C = native()
        M, K = x2.shape
        N = weight.shape[0]
        # a factored DDP weight (world size > 1): this rank's x rows are staged now and their
        # all-gather issued on the comm stream, after the GEMM below is launched
        fwd_gather = fac is not None and fac.factor_forward(weight, x2)
        if planes_fit(M, N, K) and weight.stride(1) == 1 and _al16(weight, bias):
            y = torch.empty((M, N), device=x2.device, dtype=torch.float32)
            # a hidden layer's output also leaves as planes: the next skinny GEMM's A operand
            op = torch.empty((3, M, N), device=x2.device, dtype=torch.bfloat16) \
                if relu and N % 32 == 0 else None
            C.gemm_planes(planes_of(x2), weight, y, True, bias=bias, relu=relu, out_planes=op)
            if op is not None:
                attach_planes(y, op)
        else:
            y = torch.empty((M, N), device=x2.device, dtype=torch.float32)
            C.gemm_f32(x2, weight, y, True, True, bias=bias, relu=relu)
        if fwd_gather:
            fac.factor_flush()  # the compute chain now owns the staging copy's first child
        ctx.relu = relu
        ctx.gate_in = gate_in
        ctx.params = (weight, bias)
        ctx.prev_w = prev[0] if prev else None
        ctx.save_for_backward(x2, weight, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        C = native()
        x2, weight, y = ctx.saved_tensors
        w_param, b_param = ctx.params
        if dy.dim() != 2 or dy.stride(1) != 1:
            dy = dy.contiguous()
        dx = dw = db = None
        want_db = b_param is not None and needs(ctx, 2)
        db = grad_dest(b_param) if want_db else None
        # ReLU backward: g = dy * (y > 0), one pass (g is dy itself without ReLU) -- unless the
        # consumer's input-gradient epilogue already applied this mask (idempotent either way)
        g = C.relu_bias_bwd(dy, y) if ctx.relu and not _pregated(dy, y) else dy
        fac = factor_target(w_param) if needs(ctx, 1) else None
        epi = epilogue_target(w_param) if needs(ctx, 1) and fac is None else None
        if needs(ctx, 0) and needs(ctx, 1) and fac is None and weight.shape[0] <= 16:
            # classifier head (out <= 16): input gradient (gated, + its planes for the next skinny
            # GEMM), weight and bias gradient in ONE launch (csrc/gemm_skinny.hip head_bwd). At
            # world size 1 with the fused optimizer the same kernel also applies the SGD / Adam
            # update to W (and b) in place and marks them done through note_epilogue (hand_off):
            # the reducer's bucket pass then skips them; otherwise it writes dw / db and the
            # update happens in the reducer's pass
            dx = _dx_buffer(ctx, x2)
            dw = grad_dest(w_param)
            gate = x2 if ctx.gate_in else None
            kw = {}
            if epi is not None and dw.is_contiguous() and not _tp_epilogue(epi):
                # world size 1 + fused optimizer: the kernel updates W (and b) in place
                kw = dict(backend=epi[0], w_offset=epi[1])
                be = bias_epilogue(b_param) if db is not None else None
                if be is not None:
                    kw.update(b_offset=be[1], b_span=be[2])
            ok, pl = C.head_bwd(g, x2, weight, dx, dw, db=db, gate=gate,
                                planes=planes_input_fit(dx.shape[0], dx.shape[1]), **kw)
            if ok:
                if kw:
                    hand_off(w_param, dw)
                    if "b_offset" in kw:
                        hand_off(b_param, db)
                if gate is not None:
                    _mark_gated(dx, x2)
                    prev = _prefetch_prev_g(ctx, dx)
                    if prev is not None:
                        prev.factor_flush()
                if pl is not None:
                    attach_planes(dx, pl)
                return dx, dw, db, None, None, None, None
        # a factored weight (world size > 1): its g all-gather starts now, ahead of the
        # input-gradient GEMM it then overlaps (DDP.factor_prefetch_g)
        g_pref = fac is not None and g.is_cuda and fac.factor_prefetch_g(w_param, g)
        if needs(ctx, 0):
            dx = _dx_buffer(ctx, x2)
            # dx[B, in] = g . W : A = g [M=B][K=out], B = W stored [K=out][N=in]
            # (before the weight-gradient GEMM: with an optimizer epilogue that one updates W).
            # When the input is a ReLU output (the previous fused Linear+ReLU), the epilogue
            # also applies that layer's mask (x > 0): its backward then skips its mask pass
            gate = x2 if ctx.gate_in else None
            M, K = g.shape
            # (a batch-sized g arrives with its planes from the head backward; a larger one
            # without them would pay a split pass the planes GEMM does not win back:
            # profiles/r9/tp_planes_r9.md)
            if planes_fit(M, x2.shape[1], K) and weight.stride(1) == 1 and \
                    _al16(weight, gate, dx) and (M <= 256 or has_planes(g)):
                C.gemm_planes(planes_of(g), weight, dx, False, gate=gate)
            else:
                C.gemm_f32(g, weight, dx, True, False, gate=gate)
            if gate is not None:
                _mark_gated(dx, x2)
                prev = _prefetch_prev_g(ctx, dx)
                if prev is not None:
                    if prev is not fac:
                        prev.factor_flush()
                    elif not g_pref:
                        g_pref = True
        if g_pref:
            fac.factor_flush()  # the captured fork follows the GEMM's node
        if needs(ctx, 1):
            dw = grad_dest(w_param)
            # dW[out, in] = g^T . x : A = g stored [K=batch][M=out], B = x stored [K][N=in];
            # the bias gradient (sum over the batch of g) is reduced inside the same kernel
            if fac is not None and fac.factor_submit(w_param, g, x2, dw):
                # world size > 1: the DDP bucket of W computes this rank's rows of the averaged
                # gradient from the all-gathered factors (g, x), and the averaged bias gradient
                # from the gathered g; dw / db are handed to autograd unwritten
                pass
            elif epi is not None and _tp_epilogue(epi):
                # a tensor-sharded weight (parallel/tensor_parallel.py register_fused_optimizer):
                # the same epilogue on the shard, whose gradient is complete on this rank
                be = bias_epilogue(b_param) if db is not None else None
                if epi[0].epilogue_gemm(g, x2, dw, w_param, db=db,
                                        b=b_param if be is not None else None):
                    hand_off(w_param, dw)
                    if be is not None:
                        hand_off(b_param, db)
            elif epi is not None:
                # world size 1 + fused optimizer: the epilogue updates W and its optimizer state
                # from the accumulators; the gradient itself is never written to HBM. hold: the
                # launch waits for the next layer's, and the two run as one persistent kernel
                # (the backend's end of backward runs one still held)
                be = bias_epilogue(b_param) if db is not None else None
                done = C.gemm_f32_opt(g, x2, dw, False, False, epi[0], epi[1], rowsum=db,
                                      bias_offset=be[1] if be else -1,
                                      bias_span=be[2] if be else 0, hold=_PAIR_WGRAD)
                if done:  # the epilogue ran: W (and b) were updated, their slots never written
                    hand_off(w_param, dw)
                    if be is not None:
                        hand_off(b_param, db)
            else:
                C.gemm_f32(g, x2, dw, False, False, rowsum=db)
        elif want_db:
            C.relu_bias_bwd(g, None, db)
        return dx, dw, db, None, None, None, None


def _tp_epilogue(epi) -> bool:
    """The epilogue target is a tensor-sharded wrapper (not a DDP reducer backend)."""
    return hasattr(epi[0], "epilogue_gemm")


class _LinearCpuFn(torch.autograd.Function):
    """The CPU twin of _LinearFn's gradient routing in torch math: gradients written straight
    into arena slots, the factored synchronisation of a DDP on CPU arenas (the gloo tests of that
    algorithm), and the device op's gradient-ready order (weight before bias)."""

    @staticmethod
    def forward(ctx, x2, weight, bias, relu: bool, gate_in: bool):
        y = F.linear(x2, weight, bias)
        if relu:
            y = F.relu(y)
        ctx.relu = relu
        ctx.gate_in = gate_in
        ctx.params = (weight, bias)
        ctx.save_for_backward(x2, weight, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x2, weight, y = ctx.saved_tensors
        w_param, b_param = ctx.params
        g = dy * (y > 0) if ctx.relu and not _pregated(dy, y) else dy
        dx = dw = db = None
        want_db = b_param is not None and needs(ctx, 2)
        db = grad_dest(b_param) if want_db else None
        if needs(ctx, 0):
            dx = g @ weight
            if ctx.gate_in:
                dx = dx * (x2 > 0)
                _mark_gated(dx, x2)
        fac = factor_target(w_param) if needs(ctx, 1) else None
        if needs(ctx, 1):
            dw = grad_dest(w_param)
            if fac is not None and fac.factor_submit(w_param, g, x2, dw):
                pass  # dw / db handed to autograd unwritten (see _LinearFn)
            else:
                dw.copy_(g.t() @ x2)
                if db is not None:
                    db.copy_(g.sum(0))
        elif db is not None:
            db.copy_(g.sum(0))
        return dx, dw, db, None, None


def _factor_owner(weight):
    """The DDP that factors ``weight``'s gradient synchronisation (it may gather the layer's
    input at forward time: DDP.factor_forward), else None."""
    ref = getattr(weight, "_tdp_factor", None)
    return ref() if ref is not None else None


def linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None,
           relu: bool = False) -> torch.Tensor:
    """``relu?(x @ weight.T + bias)`` for x of shape [..., in_features]."""
    # the input is the ReLU output of a previous fused Linear(+ReLU): this layer's input-gradient
    # epilogue applies that ReLU's mask (see _LinearFn.backward)
    gate_in = bool(getattr(x, "_tdp_relu_out", False)) and x.dim() == 2
    if not x.is_cuda:
        if torch.is_grad_enabled() and x.dtype == torch.float32:
            # the device op's gradient routing (arena slots, factored sync, hook order) in torch
            # math: the CPU/gloo tests see the same parameter-ready order as MI355X
            note_use(weight)
            lead = x.shape[:-1]
            y = _LinearCpuFn.apply(x.reshape(-1, x.shape[-1]), weight, bias, relu, gate_in)
            if relu and x.dim() == 2:
                y._tdp_relu_out = True
            return y if x.dim() == 2 else y.reshape(*lead, weight.shape[0])
        y = F.linear(x, weight, bias)
        return F.relu(y) if relu else y
    if x.dtype != torch.float32:
        raise TypeError(f"native linear expects float32 activations, got {x.dtype}")
    lead = x.shape[:-1]
    x2 = x if x.dim() == 2 else x.reshape(-1, x.shape[-1])
    if x2.stride(-1) != 1:
        x2 = x2.contiguous()
        gate_in = False
    if torch.is_grad_enabled():
        note_use(weight)
    fac = _factor_owner(weight) if torch.is_grad_enabled() else None
    # the weight that produced x (a fused Linear+ReLU before this one): its g is this layer's
    # gated dx, whose gather this layer's backward can start (a tuple: not an autograd input)
    pw = getattr(x, "_tdp_prod_w", None) if gate_in else None
    y = _LinearFn.apply(x2, weight, bias, relu, gate_in, fac, (pw,) if pw is not None else None)
    if x.dim() == 2:
        if relu:
            y._tdp_relu_out = True
            y._tdp_prod_w = weight
        return y
    return y.reshape(*lead, weight.shape[0])
