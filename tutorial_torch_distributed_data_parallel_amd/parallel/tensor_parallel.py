"""Tensor-sharded execution of the toy MLP with data-parallel training semantics.

What the reference does: ``DDP(model)`` (/root/reference/multi-GPU-training-torch.py:245), then
per step ``loss.backward()`` -- every rank all-reduces the full 218 MB gradient -- and
``optimizer.step()`` on a full replica (:125-126). Same math here, different execution: the
hidden Linear pair is split Megatron-style over the W ranks of the node, so what crosses xGMI
each step is ACTIVATIONS (a few MB), not weights:

  X   = every rank's batch, in rank order           [W*B, in]      (gathered from the rank's
        own dataset replica with global_batch=True -- bench.py -- else all-gathered)
  H1  = relu?(X . W1[own rows]^T + b1[own])         [W*B, h1/W]    column-parallel fc1
        (BatchNorm1d here sees the GLOBAL batch: SyncBN statistics with no collective)
  P2  = H1 . W2[:, own cols]^T                      [W*B, h2]      row-parallel fc2 (partial)
  H2  = relu?(reduce_scatter_rows(P2) + b2)         [B, h2]        this rank's samples
  out = fc3(H2)                                     [B, classes]   replicated head

Backward is autograd through the same ops: the reduce-scatter's gradient is the all-gather of
dH2, scaled by 1/W (folded into the bias + ReLU backward pass) so that every sharded gradient is
the global-batch MEAN that DDP's averaged all-reduce produces; the replicated parameters (b2,
the head, a BatchNorm after fc2) get the usual averaged all-reduce (~0.2 MB). Each rank then
updates only its shard with the ordinary optimizer: 1/W of the optimizer's HBM traffic, the
dominant cost of the dp1 step (profiles/r9/wgrad_split_roles_r9.md).

Streams (GPU, W > 1): the backward all-gather and then the replicated all-reduce run on a
communication stream (the all-reduce behind the gradient GEMMs); fc2's weight-gradient GEMM runs
on an auxiliary stream beside fc1's, which has fewer tiles than workgroup slots; both are joined
in ``sync_grads``. ``overlap_chunks`` > 1 splits fc2's reduce-scatter / all-gather into column
chunks behind the chunk GEMMs. Captured into the step's hipGraph like everything else.

Per step and rank at W ranks, B samples each (toy MLP 9216-4096-4096-10, fp32): X all-gather
(W-1) B 9216 x 4 B (33 MB at W = 8), reduce-scatter and all-gather of [W*B, 4096] (2 x 14.7 MB
at W = 8) -- against (W-1)/W x 218 MB x 2 for a gradient all-reduce or the factored modes'
parameter all-gathers (parallel/commmodel.py, docs/COMM_MODEL.md "Tensor-sharded"). GEMM work
per rank equals dp1's; numerics are fp32 (the same kernels), summation order differs from the
replicated step (tests/test_tensor_parallel_cpu.py checks the step against the one-process
global-batch step).

``state_dict()`` of the wrapper is the full model's (rank-order all-gathers), so checkpoints
stay those of the unsharded ToyMLP (utils/checkpoint.py).
"""
from __future__ import annotations

import contextlib
import weakref

import torch
import torch.distributed as dist
import torch.nn as nn

from . import runtime
from .arena import ParamArena
from ..nn import BatchNorm1d, Linear, SyncBatchNorm


# Measurement only (scripts/tp_rank_proxy.py): one process plays rank 0 of a W-rank job -- shard
# shapes of W ranks, every collective replaced by its local copy (no peer traffic): the per-rank
# compute of the W-rank step on one GPU.
_FAKE_WORLD = 0


def set_fake_world(w: int) -> None:
    global _FAKE_WORLD
    _FAKE_WORLD = int(w)


def _ranks():
    if _FAKE_WORLD:
        return 0, _FAKE_WORLD
    return runtime.get_rank(), runtime.get_world_size()


def _all_gather_rows(out: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """out[r*n:(r+1)*n] = rank r's x (ordered on the current stream on the GPU)."""
    rank, world = _ranks()
    if world == 1:
        out.copy_(x)
        return out
    if _FAKE_WORLD:
        out.view((world,) + tuple(x.shape)).copy_(x.unsqueeze(0).expand((world,) + tuple(x.shape)))
        return out
    comm = runtime.comm()
    if x.is_cuda and comm is not None:
        comm.all_gather(out, x.contiguous())
    else:
        dist.all_gather(list(out.chunk(world)), x.contiguous())
    return out


def _reduce_scatter_rows(out: torch.Tensor, p: torch.Tensor) -> torch.Tensor:
    """out = sum over ranks of rank r's p[rank*n:(rank+1)*n] (this rank's row block)."""
    rank, world = _ranks()
    if world == 1 or _FAKE_WORLD:
        out.copy_(p[: out.shape[0]])
        return out
    comm = runtime.comm()
    if p.is_cuda and comm is not None:
        comm.reduce_scatter(out, p.contiguous(), "sum")
    else:  # gloo has no reduce-scatter: all-reduce, keep the own block
        full = p.contiguous().clone()
        dist.all_reduce(full)
        out.copy_(full.chunk(world)[rank])
    return out


class _GatherRows(torch.autograd.Function):
    """Every rank's rows, in rank order; the gradient of this rank's rows is the sum over ranks
    of their gradient blocks (a reduce-scatter)."""

    @staticmethod
    def forward(ctx, x):
        _, world = _ranks()
        out = torch.empty((world * x.shape[0],) + tuple(x.shape[1:]), device=x.device,
                          dtype=x.dtype)
        return _all_gather_rows(out, x)

    @staticmethod
    def backward(ctx, dy):
        _, world = _ranks()
        out = torch.empty((dy.shape[0] // world,) + tuple(dy.shape[1:]), device=dy.device,
                          dtype=dy.dtype)
        return _reduce_scatter_rows(out, dy)


class _RowParallelOverlap(torch.autograd.Function):
    """fc2 of the sharded pair: ``reduce_scatter_rows(h1 . w2^T)``, in ``nc`` column chunks of
    fc2's output when nc > 1 (chunk c's GEMM on the compute stream while chunk c-1's
    reduce-scatter runs on the communication stream; nc = 1: one GEMM, the reduce-scatter on
    the compute stream). Backward: the all-gather(s) of dY (times ``scale``) on the
    communication stream; dW2 = dP^T H1 on an auxiliary stream, so its GEMMs fill the CUs that
    fc1's weight-gradient GEMM (fewer tiles than slots: 288 for 512 at W = 8) leaves idle (joined
    in ``sync_grads``); dH1 = dP W2 on the compute stream, gated by fc1's ReLU in its epilogue
    when fc1's output is one (fc1's backward then skips its mask pass). On CPU the same chunk
    loop runs without streams (the gloo tests of the indexing)."""

    @staticmethod
    def forward(ctx, h1, w2, scale: float, nc: int, side, owner=None):
        from .._native import native

        _, world = _ranks()
        M, s = h1.shape
        h2 = w2.shape[0]
        hc = h2 // nc
        B = M // world
        parts = torch.empty((nc, B, hc), device=h1.device, dtype=h1.dtype)
        ctx.save_for_backward(h1, w2)
        ctx.scale, ctx.nc, ctx.side, ctx.owner = scale, nc, side, owner
        ctx.gate = bool(getattr(h1, "_tdp_relu_out", False)) and h1.is_cuda
        if not h1.is_cuda:
            for c in range(nc):
                _reduce_scatter_rows(parts[c], h1 @ w2[c * hc:(c + 1) * hc].t())
            return parts.transpose(0, 1).reshape(B, h2)
        from ..ops._grad import note_use
        from ..ops.linear import planes_fit, planes_of

        note_use(w2)  # the fused optimizer's epilogue needs exactly one use per step
        C = native()
        hp = planes_of(h1) if planes_fit(M, hc, s) else None

        def chunk(c, out):
            if hp is not None:  # H1's pre-split planes (fc1's epilogue emitted them)
                C.gemm_planes(hp, w2[c * hc:(c + 1) * hc], out, True)
            else:
                C.gemm_f32(h1, w2[c * hc:(c + 1) * hc], out, True, True)
        if nc == 1:
            pc = torch.empty((M, h2), device=h1.device, dtype=h1.dtype)
            chunk(0, pc)
            return _reduce_scatter_rows(parts[0], pc)
        if side is None:  # no communication stream (local-copy measurement): in order
            for c in range(nc):
                pc = torch.empty((M, hc), device=h1.device, dtype=h1.dtype)
                chunk(c, pc)
                _reduce_scatter_rows(parts[c], pc)
            return parts.transpose(0, 1).reshape(B, h2)
        comp = torch.cuda.current_stream()
        keep = []
        for c in range(nc):
            pc = torch.empty((M, hc), device=h1.device, dtype=h1.dtype)
            chunk(c, pc)
            ev = torch.cuda.Event()
            ev.record(comp)
            side.wait_event(ev)
            with torch.cuda.stream(side):
                _reduce_scatter_rows(parts[c], pc)
            keep.append(pc)  # alive until the join below orders their reuse after it
        done = torch.cuda.Event()
        done.record(side)
        comp.wait_event(done)
        del keep
        return parts.transpose(0, 1).reshape(B, h2)

    @staticmethod
    def backward(ctx, dy):
        from .._native import native
        from ..ops._grad import epilogue_target, grad_dest, hand_off
        from ..ops.linear import _mark_gated

        h1, w2 = ctx.saved_tensors
        nc, scale, side, owner = ctx.nc, ctx.scale, ctx.side, ctx.owner
        _, world = _ranks()
        M, s = h1.shape
        h2 = w2.shape[0]
        hc = h2 // nc
        B = dy.shape[0]
        # this rank's rows of dY, scaled, chunk-major: [nc][B][hc]
        dyc = (dy * scale if scale != 1.0 else dy).reshape(B, nc, hc).transpose(0, 1).contiguous()
        dp = torch.empty((nc, M, hc), device=dy.device, dtype=dy.dtype)
        dh1 = torch.empty_like(h1) if ctx.needs_input_grad[0] else None
        dw2 = grad_dest(w2) if ctx.needs_input_grad[1] else None
        if not dy.is_cuda:
            for c in range(nc):
                _all_gather_rows(dp[c], dyc[c])
                if dw2 is not None:
                    dw2[c * hc:(c + 1) * hc].copy_(dp[c].t() @ h1)
                if dh1 is not None:
                    t = dp[c] @ w2[c * hc:(c + 1) * hc]
                    dh1.copy_(t) if c == 0 else dh1.add_(t)
            return dh1, dw2, None, None, None, None
        C = native()
        comp = torch.cuda.current_stream()
        side = owner.comm_stream() if owner is not None else side
        aux = owner.aux_stream() if owner is not None else None
        ready = torch.cuda.Event()
        ready.record(comp)
        evs = []
        if side is not None:
            side.wait_event(ready)
            with torch.cuda.stream(side):
                for c in range(nc):
                    _all_gather_rows(dp[c], dyc[c])
                    e = torch.cuda.Event()
                    e.record(side)
                    evs.append(e)
                if owner is not None:
                    owner._reduce_replicated_async()
        else:
            for c in range(nc):
                _all_gather_rows(dp[c], dyc[c])
            ready = torch.cuda.Event()  # the gathered dP (compute stream) for the aux stream
            ready.record(comp)
        if owner is not None:
            owner._keep += [dyc, dp, h1]
        if dh1 is not None:
            for c in range(nc):
                if evs:
                    comp.wait_event(evs[c])
                last = c == nc - 1
                # dH1 (+)= dP_c . W2[rows of chunk c]; the last chunk's epilogue applies fc1's
                # ReLU mask to the finished sum
                C.gemm_f32(dp[c], w2[c * hc:(c + 1) * hc], dh1, True, False,
                           beta=0.0 if c == 0 else 1.0, gate=h1 if (ctx.gate and last) else None)
            if ctx.gate:
                _mark_gated(dh1, h1)
        # the fused optimizer (register_fused_optimizer): each chunk's epilogue updates its rows
        # of W2 in place instead of writing the gradient
        epi = epilogue_target(w2) if dw2 is not None else None
        handed = []

        def dw2_chunk(c):
            out = dw2[c * hc:(c + 1) * hc]
            if epi is not None and epi[0].epilogue_gemm(dp[c], h1, out, w2, row0=c * hc):
                handed.append(c)
            else:
                C.gemm_f32(dp[c], h1, out, False, False)
        if dw2 is not None:
            if aux is not None and w2.grad is None:
                # (only into W2's arena slot: a fresh gradient tensor -- accumulation -- goes
                # straight to autograd's AccumulateGrad on the compute stream, so it is computed
                # there)
                # dW2[rows of chunk c] = dP_c^T . H1 on the aux stream, released only once dH1
                # is done: it then runs beside fc1's weight-gradient GEMM (next on the compute
                # stream, fewer tiles than slots) instead of competing with dH1 for the CUs
                after_dh1 = torch.cuda.Event()
                after_dh1.record(comp)
                with torch.cuda.stream(aux):
                    aux.wait_event(after_dh1)
                    for c in range(nc):
                        dw2_chunk(c)
                    done = torch.cuda.Event()
                    done.record(aux)
                owner._aux_done = done
            else:
                for c in range(nc):
                    if evs:
                        comp.wait_event(evs[c])
                    dw2_chunk(c)
            if handed:
                hand_off(w2, dw2)
        return dh1, dw2, None, None, None, None


class _BiasReLU(torch.autograd.Function):
    """``relu?(y + b)`` for the reduce-scattered fc2 output, one native pass each way: forward
    csrc bias_act, backward relu_bias_bwd (the ReLU mask, the bias gradient into b's arena slot,
    and the input gradient times ``gscale`` -- the 1/W of the sharded gradients, folded here
    instead of a separate scaling pass; the bias gradient itself stays unscaled)."""

    @staticmethod
    def forward(ctx, y, b, relu: bool, gscale: float = 1.0):
        if y.is_cuda:
            from .._native import native

            out = native().bias_act(y, b, relu)
        else:
            out = y + b
            if relu:
                out.clamp_min_(0.0)
        ctx.relu, ctx.gscale = relu, gscale
        ctx.b = b
        ctx.save_for_backward(out if relu else None)
        return out

    @staticmethod
    def backward(ctx, dy):
        from .._native import native
        from ..ops._grad import grad_dest

        (out,) = ctx.saved_tensors
        db = grad_dest(ctx.b) if ctx.needs_input_grad[1] else None
        if dy.is_cuda:
            dy = dy.contiguous()
            if ctx.relu:
                g = native().relu_bias_bwd(dy, out, db, gscale=ctx.gscale)
            elif db is not None:
                g = native().relu_bias_bwd(dy, None, db)
                g = g * ctx.gscale if ctx.gscale != 1.0 else g
            else:
                g = dy * ctx.gscale if ctx.gscale != 1.0 else dy
        else:
            g = dy * (out > 0) if ctx.relu else dy
            if db is not None:
                db.copy_(g.sum(0))
            if ctx.gscale != 1.0:
                g = g * ctx.gscale
        return g, db, None, None


def _linears(model):
    order = getattr(model, "_order", None)
    if order is None:
        raise TypeError("TensorParallelMLP: expects a ToyMLP-like module (an ordered stack of "
                        "Linear [+ BatchNorm1d] layers)")
    mods = [(n, getattr(model, n)) for n in order]
    return mods


class TensorParallelMLP(nn.Module):
    """Wrap a (full, identically initialised) ToyMLP with two hidden layers for tensor-sharded
    training at the current world size; ``forward`` takes this rank's batch and returns this
    rank's logits, exactly like ``DDP(model)(x)``. Call ``sync_grads()`` after backward (the
    averaged all-reduce of the replicated parameters' gradients), then ``optimizer.step()`` on
    ``parameters()``.

    ``global_batch=True``: ``forward`` receives the whole node's batch [W*B, in] in rank order
    (every rank gathered it from its replica of the dataset) and skips the input all-gather."""

    def __init__(self, model: nn.Module, global_batch: bool = False, overlap_chunks: int = 1):
        super().__init__()
        self.overlap_chunks = int(overlap_chunks)
        rank, world = _ranks()
        self.rank, self.world = rank, world
        self.global_batch = bool(global_batch)
        mods = _linears(model)
        lin = [(n, m) for n, m in mods if isinstance(m, nn.Linear)]
        bns = {n: m for n, m in mods if isinstance(m, nn.modules.batchnorm._BatchNorm)}
        if len(lin) != 3:
            raise ValueError("TensorParallelMLP: supports the toy MLP's shape (two hidden "
                             f"Linear layers and a head), got {len(lin)} Linear layers")
        (n1, fc1), (n2, fc2), (n3, fc3) = lin
        h1 = fc1.out_features
        if h1 % world or (h1 // world) % 4:
            raise ValueError(f"TensorParallelMLP: hidden width {h1} must split into W = "
                             f"{world} shards of a multiple of 4")
        names = [n for n, _ in mods]
        bn1 = bns.get(names[names.index(n1) + 1]) if names.index(n1) + 1 < len(names) else None
        bn2 = bns.get(names[names.index(n2) + 1]) if names.index(n2) + 1 < len(names) else None
        if bn1 is not None and world > 1 and not isinstance(bn1, SyncBatchNorm):
            raise ValueError("TensorParallelMLP: the BatchNorm after fc1 normalises over the "
                             "node's batch here (SyncBN statistics); per-rank statistics "
                             "(plain BatchNorm1d) are not supported -- convert_sync_batchnorm")
        # every shard is cut from rank 0's weights (DDP's construction-time broadcast)
        with torch.no_grad():
            for t in list(model.parameters()) + list(model.buffers()):
                runtime.broadcast(t.data, 0)
        self._names = (n1, n2, n3)
        self._bn_names = (names[names.index(n1) + 1] if bn1 is not None else None,
                          names[names.index(n2) + 1] if bn2 is not None else None)
        self._dims = (fc1.in_features, h1, fc2.out_features, fc3.out_features)
        self._side = None  # communication stream (comm_stream)
        self._reduced = None  # event: the replicated all-reduce issued from the backward
        self._keep = []  # tensors read on the communication stream, alive until the join
        self._fresh = False
        self._aux = None  # auxiliary stream (aux_stream)
        self._aux_done = None  # event: fc2's weight-gradient GEMMs on it
        if fc2.out_features % max(1, self.overlap_chunks) or (fc2.weight.is_cuda and (
                fc2.out_features // max(1, self.overlap_chunks)) % 4):
            raise ValueError(f"TensorParallelMLP: fc2 width {fc2.out_features} does not split "
                             f"into {self.overlap_chunks} chunks of a multiple of 4")
        s = h1 // world
        lo, hi = rank * s, (rank + 1) * s
        dev = fc1.weight.device
        with torch.no_grad():
            relu1 = bn1 is None
            self.fc1 = Linear(fc1.in_features, s, bias=fc1.bias is not None, relu=relu1,
                              device=dev)
            self.fc1.weight.copy_(fc1.weight[lo:hi])
            if fc1.bias is not None:
                self.fc1.bias.copy_(fc1.bias[lo:hi])
            self.bn1 = None
            if bn1 is not None:
                self.bn1 = BatchNorm1d(s, eps=bn1.eps, momentum=bn1.momentum,
                                       affine=bn1.affine,
                                       track_running_stats=bn1.track_running_stats,
                                       relu=getattr(bn1, "relu", False), device=dev)
                for name in ("weight", "bias", "running_mean", "running_var"):
                    src = getattr(bn1, name, None)
                    if src is not None:
                        getattr(self.bn1, name).copy_(src[lo:hi])
                if bn1.num_batches_tracked is not None:
                    self.bn1.num_batches_tracked.copy_(bn1.num_batches_tracked)
                self.bn1._nbt = getattr(bn1, "_nbt", 0)
            self.fc2 = Linear(s, fc2.out_features, bias=False, device=dev)
            self.fc2.weight.copy_(fc2.weight[:, lo:hi])
            self.b2 = nn.Parameter(fc2.bias.detach().clone()) if fc2.bias is not None else None
            self.relu2 = bn2 is None and getattr(fc2, "relu", False)
            self.bn2 = bn2  # replicated: normalises this rank's rows (sync or not, as given)
            self.fc3 = fc3
        self._replicated = [p for p in ([self.b2] if self.b2 is not None else [])] + \
            (list(bn2.parameters()) if bn2 is not None else []) + list(fc3.parameters())
        # one flat arena, replicated parameters first: their gradients are ONE contiguous range
        # (a single all-reduce, no packing), every gradient has its slot (the optimizer's
        # single-kernel, capture-safe flat step: optim/fused.py)
        rep = {id(q) for q in self._replicated}
        self._arena = ParamArena(self._replicated +
                                 [q for q in self.parameters() if id(q) not in rep])
        last = len(self._replicated) - 1
        self._rep_end = self._arena.offsets[last] + self._arena.numels[last]
        self._index = {id(q): i for i, q in enumerate(self._arena.params)}
        self._fopt = None     # optimizer applied in the shards' weight-gradient GEMM epilogues
        self._fstate = None   # (momentum arena or None, hyper block, param group) of this step
        self._uses = {}       # forward uses per parameter (an epilogue needs exactly one)
        self._done = {}       # arena index -> elements the epilogues updated in this step
        self._epi_on = True   # off inside no_sync()

    # ---------------------------------------------------------------------------- forward
    def forward(self, x):
        # every replicated gradient is empty: this backward writes them into their arena slots
        # (ops/_grad.py grad_dest), so the backward may all-reduce the slots early
        ev = self._reduced
        if ev is not None:
            # an earlier backward of this accumulation already all-reduced its replicated
            # gradients (on the communication stream): order this pass's accumulation after it;
            # sync_grads then reduces the sum again (averaging averaged values is exact)
            torch.cuda.current_stream().wait_event(ev)
            self._reduced = None
        if self._aux_done is not None:
            # an earlier backward of this accumulation computed fc2's weight gradient on the
            # aux stream; this pass's AccumulateGrad adds into it on the compute stream, so
            # the compute stream waits for it (the event stays for sync_grads)
            torch.cuda.current_stream().wait_event(self._aux_done)
        self._fresh = self._epi_on and all(q.grad is None for q in self._replicated)
        if self._fopt is not None and torch.is_grad_enabled() and self.training:
            if self._fstate is None:  # once per optimizer step (accumulation: several forwards)
                self._begin_fused_step()
            self._uses = {}
        x = x.reshape(x.shape[0], -1)
        X = x if (self.world == 1 or self.global_batch) else _GatherRows.apply(x)
        h = self.fc1(X)
        if self.bn1 is not None:
            h = self.bn1(h)
        nc = self.overlap_chunks
        # the 1/W of the sharded gradients: folded into the bias + ReLU backward when there is
        # one (no separate scaling pass), else applied before the backward all-gather
        inv = 1.0 / self.world
        fold = self.world > 1 and self.b2 is not None
        if self.world > 1:
            y = _RowParallelOverlap.apply(h, self.fc2.weight, 1.0 if fold else inv, nc,
                                          self.comm_stream() if nc > 1 else None, self)
        else:
            y = self.fc2(h)
        if self.b2 is not None:
            y = _BiasReLU.apply(y, self.b2, self.relu2, inv if fold else 1.0)
        elif self.relu2:
            y = torch.relu(y)
        if self.bn2 is not None:
            y = self.bn2(y)
        return self.fc3(y)

    def comm_stream(self):
        """The communication stream (GPU, W > 1): fc2's overlapped collectives, the backward
        all-gather and the replicated gradients' all-reduce; created on first use."""
        if self.world == 1 or _FAKE_WORLD or not self.fc1.weight.is_cuda:
            return None
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.fc1.weight.device, priority=-1)
        return self._side

    def aux_stream(self):
        """A second side stream (GPU, W > 1) for fc2's weight-gradient GEMMs, which run beside
        fc1's backward; joined in ``sync_grads``."""
        if self.world == 1 or not self.fc1.weight.is_cuda:
            return None
        if self._aux is None:
            self._aux = torch.cuda.Stream(device=self.fc1.weight.device)
        return self._aux

    def _reduce_replicated_async(self) -> None:
        """(On the communication stream, from the backward:) the replicated parameters'
        averaged all-reduce; ``sync_grads`` joins it."""
        if not self._fresh:
            # gradients accumulate across backward passes (no zero_grad(set_to_none=True)):
            # autograd adds this pass's into .grad after this node -- sync_grads reduces them
            return
        a = self._arena
        runtime.all_reduce(a.grad[: self._rep_end], "avg")
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        self._reduced = ev

    def sync_grads(self) -> None:
        """Every gradient into its arena slot (a gradient autograd produced elsewhere is copied
        in), then the averaged all-reduce of the replicated parameters' gradients: one
        collective over the arena's leading range -- already issued from the backward on the
        communication stream (joined here), or run here."""
        a = self._arena
        ev, self._reduced = self._reduced, None
        if ev is not None:
            torch.cuda.current_stream().wait_event(ev)
        aux, self._aux_done = self._aux_done, None
        if aux is not None:
            torch.cuda.current_stream().wait_event(aux)
        # the compute stream is ordered after every side-stream read of these (the gathered
        # event, or the join above): their memory may be reused from here on
        self._keep.clear()
        late = False  # a replicated gradient that was not in its slot at the early all-reduce
        with torch.no_grad():
            for i, q in enumerate(a.params):
                if q.grad is not None and not a.is_arena_grad(i):
                    g = a.grad_view(i)
                    g.copy_(q.grad)
                    q.grad = g
                    late = late or a.offsets[i] < self._rep_end
        if self.world == 1 or _FAKE_WORLD or (ev is not None and not late):
            return
        # (after an early all-reduce: averaging the already-averaged slots again leaves every
        # rank with identical values, and the late gradient gets its average)
        runtime.all_reduce(a.grad[: self._rep_end], "avg")

    # ------------------------------------------------------------------ fused optimizer
    def register_fused_optimizer(self, optimizer) -> bool:
        """Apply ``optimizer`` to the SHARDED weights inside their weight-gradient GEMMs: the
        epilogue reads p and the momentum at each gradient element, updates them and never
        writes the gradient (csrc/gemm_f32_fast.hip OptEpilogue). A shard's gradient is complete
        on its own rank -- nothing is reduced before the update -- so this holds at any world
        size, where DDP can do it at world size 1 only (parallel/ddp.py register_fused_optimizer).
        ``optimizer.step()`` then updates what no epilogue did: the replicated parameters after
        their all-reduce, BatchNorm shards, a weight whose GEMM plan has no epilogue. Saves the
        gradient's HBM write and re-read and the separate update pass (per-rank compute at W = 2:
        391 -> 342 us, profiles/r9/tp_fused_r9ak.md). tdp SGD, one parameter group over ``parameters()``, GPU; returns
        False and changes nothing otherwise. Each backward applies the update: run the earlier
        passes of a gradient accumulation under ``no_sync()``."""
        from ..optim.fused import SGD

        if not self.fc1.weight.is_cuda or not isinstance(optimizer, SGD) or \
                len(optimizer.param_groups) != 1:
            return False
        g = optimizer.param_groups[0]
        if {id(q) for q in g["params"]} != set(self._index) or g["grad_scale"] != 1.0:
            return False
        self._fopt = optimizer
        optimizer._fused_tp = weakref.ref(self)
        me = weakref.ref(self)
        for q in (self.fc1.weight, self.fc1.bias, self.fc2.weight):
            if q is not None:
                q._tdp_epi = me
        return True

    @contextlib.contextmanager
    def no_sync(self):
        """Gradient accumulation (DDP.no_sync): backward passes inside neither all-reduce the
        replicated gradients early nor apply the fused update -- they store their gradients,
        which autograd accumulates; the pass after it accumulates too and leaves the whole update
        to ``sync_grads()`` + ``optimizer.step()``."""
        prev, self._epi_on = self._epi_on, False
        try:
            yield
        finally:
            self._epi_on = prev

    def _begin_fused_step(self) -> None:
        """(forward, before any epilogue of this step:) the momentum arena, the device hyper
        block with the current scalars, and the block's per-step advance (first-step flag)."""
        from .._native import native

        opt, a = self._fopt, self._arena
        g = opt.param_groups[0]
        buf, fresh = None, False
        if g["momentum"] != 0:
            bufs, fresh = opt._flat_state(a, ("momentum_buffer",))
            buf = bufs["momentum_buffer"]
        if 0 in opt._blocks:
            blk = opt._blocks[0][0]
            opt.sync_hyper()
            if fresh:
                opt._request_first(blk)
        else:
            blk = opt.hyper_block(0, device=self.fc1.weight.device, first=fresh)
        native().opt_step_begin(blk, 1)
        self._fstate = (buf, blk, g)
        self._done = {}

    def _note_use(self, p) -> None:  # ops/_grad.py note_use
        self._uses[id(p)] = self._uses.get(id(p), 0) + 1

    def epilogue_slot(self, p):  # ops/_grad.py epilogue_target
        if self._fstate is None or not self._epi_on or self._uses.get(id(p), 0) != 1:
            return None
        return self, self._index[id(p)]

    def bias_epilogue(self, b):  # ops/_grad.py bias_epilogue
        if self._fstate is None or not self._epi_on or id(b) not in self._index:
            return None
        return self, self._index[id(b)], None

    def note_handed(self, p, t) -> None:  # ops/_grad.py hand_off: tracked in epilogue_gemm
        pass

    def epilogue_gemm(self, A, B, C, w, row0: int = 0, db=None, b=None) -> bool:
        """C = A^T B (both MN-contiguous: the weight-gradient layout) for rows ``row0 ..`` of the
        sharded weight ``w``, with SGD applied to those rows in the epilogue (and to the bias
        ``b`` from the row sums ``db``). False: the plan had no epilogue, C / db hold the
        gradient and ``optimizer.step()`` updates them."""
        from .._native import native

        buf, blk, g = self._fstate
        a = self._arena
        i = self._index[id(w)]
        n = C.numel()
        start = a.offsets[i] + row0 * C.shape[1]
        bp = bb = None
        if b is not None and db is not None:
            j = self._index[id(b)]
            bo = a.offsets[j]
            bp = a.data[bo:bo + b.numel()]
            bb = buf[bo:bo + b.numel()] if buf is not None else None
        done = native().gemm_f32_sgd(A, B, C, False, False, a.data[start:start + n],
                                     buf[start:start + n] if buf is not None else None, blk,
                                     nesterov=g["nesterov"], maximize=g["maximize"], rowsum=db,
                                     bias_p=bp, bias_buf=bb)
        if done:
            self._done[i] = self._done.get(i, 0) + n
            if bp is not None:
                self._done[j] = a.numels[j]
        return done

    def _fused_step(self, opt) -> None:
        """``optimizer.step()`` with the fused optimizer: one flat update per run of arena
        parameters no epilogue updated (gradients in their slots: sync_grads ran)."""
        from .._native import native

        if self._fstate is None:
            self._begin_fused_step()
        buf, blk, g = self._fstate
        a = self._arena
        spans = []
        for i in range(len(a.params)):
            done = self._done.get(i, 0)
            if done == a.numels[i] or a.params[i].grad is None:
                continue
            if done:
                raise RuntimeError("tensor-sharded fused optimizer: a weight was updated in part")
            end = a.offsets[i + 1] if i + 1 < len(a.params) else a.numel
            if spans and spans[-1][1] == a.offsets[i]:
                spans[-1][1] = end
            else:
                spans.append([a.offsets[i], end])
        C = native()
        for lo, hi in spans:
            C.sgd_flat(a.data[lo:hi], a.grad[lo:hi], buf[lo:hi] if buf is not None else None,
                       g["lr"], g["momentum"], g["dampening"], g["weight_decay"], g["nesterov"],
                       g["maximize"], False, 1.0, hyper=blk)
        self._fstate = None
        self._done = {}

    def check_replicas(self) -> None:
        """Raise unless every rank holds bit-identical replicated parameters (collective)."""
        if self.world == 1 or _FAKE_WORLD:
            return
        flat = torch.cat([p.detach().reshape(-1) for p in self._replicated])
        out = torch.empty(self.world * flat.numel(), device=flat.device, dtype=flat.dtype)
        _all_gather_rows(out, flat)
        for r, part in enumerate(out.chunk(self.world)):
            if not torch.equal(part, flat):
                raise RuntimeError(f"tensor-sharded step: replicated parameters of rank {r} "
                                   f"differ from rank {self.rank}'s")

    # ----------------------------------------------------------------------- checkpoints
    def _gather_rows(self, t: torch.Tensor) -> torch.Tensor:
        if self.world == 1:
            return t.detach().clone()
        out = torch.empty((self.world * t.shape[0],) + tuple(t.shape[1:]), device=t.device,
                          dtype=t.dtype)
        return _all_gather_rows(out, t.detach().contiguous())

    def full_state_dict(self) -> dict:
        """The unsharded ToyMLP state_dict (collective: every rank must call it)."""
        n1, n2, n3 = self._names
        b1n, b2n = self._bn_names
        sd = {f"{n1}.weight": self._gather_rows(self.fc1.weight)}
        if self.fc1.bias is not None:
            sd[f"{n1}.bias"] = self._gather_rows(self.fc1.bias)
        if self.bn1 is not None:
            for k, v in self.bn1.state_dict().items():
                sd[f"{b1n}.{k}"] = v.clone() if k == "num_batches_tracked" else \
                    self._gather_rows(v)
        # fc2 columns: gather the [h2, s] shards as rows of their transposes
        sd[f"{n2}.weight"] = self._gather_rows(self.fc2.weight.t().contiguous()).t().contiguous()
        if self.b2 is not None:
            sd[f"{n2}.bias"] = self.b2.detach().clone()
        if self.bn2 is not None:
            for k, v in self.bn2.state_dict().items():
                sd[f"{b2n}.{k}"] = v.clone()
        for k, v in self.fc3.state_dict().items():
            sd[f"{n3}.{k}"] = v.clone()
        return sd

    def state_dict(self, *args, **kwargs):  # noqa: D401 - the full model's (collective)
        """The unsharded ToyMLP state_dict, every rank must call it (all-gathers): checkpoints
        of the tensor-sharded job are those of the replicated model (utils/checkpoint.py)."""
        if args or kwargs.get("destination") is not None or kwargs.get("prefix"):
            return super().state_dict(*args, **kwargs)  # nn.Module internals: local shards
        return self.full_state_dict()

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        """Load an unsharded ToyMLP state_dict (this rank keeps its slices)."""
        n1, n2, n3 = self._names
        want = set(self.full_state_dict_keys())
        missing = sorted(want - set(state_dict))
        unexpected = sorted(set(state_dict) - want)
        if strict and (missing or unexpected):
            raise RuntimeError(f"TensorParallelMLP.load_state_dict: missing {missing}, "
                               f"unexpected {unexpected}")
        self.load_full_state_dict(state_dict)
        from torch.nn.modules.module import _IncompatibleKeys

        return _IncompatibleKeys(missing, unexpected)

    def full_state_dict_keys(self):
        n1, n2, n3 = self._names
        b1n, b2n = self._bn_names
        keys = [f"{n1}.weight"] + ([f"{n1}.bias"] if self.fc1.bias is not None else [])
        if self.bn1 is not None:
            keys += [f"{b1n}.{k}" for k in self.bn1.state_dict()]
        keys += [f"{n2}.weight"] + ([f"{n2}.bias"] if self.b2 is not None else [])
        if self.bn2 is not None:
            keys += [f"{b2n}.{k}" for k in self.bn2.state_dict()]
        keys += [f"{n3}.{k}" for k in self.fc3.state_dict()]
        return keys

    def load_full_state_dict(self, sd: dict) -> None:
        n1, n2, n3 = self._names
        b1n, b2n = self._bn_names
        s = self._dims[1] // self.world
        lo, hi = self.rank * s, (self.rank + 1) * s
        with torch.no_grad():
            self.fc1.weight.copy_(sd[f"{n1}.weight"][lo:hi])
            if self.fc1.bias is not None:
                self.fc1.bias.copy_(sd[f"{n1}.bias"][lo:hi])
            if self.bn1 is not None:
                for k, v in self.bn1.state_dict().items():
                    src = sd[f"{b1n}.{k}"]
                    v.copy_(src if k == "num_batches_tracked" else src[lo:hi])
            self.fc2.weight.copy_(sd[f"{n2}.weight"][:, lo:hi])
            if self.b2 is not None:
                self.b2.copy_(sd[f"{n2}.bias"])
            if self.bn2 is not None:
                self.bn2.load_state_dict({k[len(b2n) + 1:]: v for k, v in sd.items()
                                          if k.startswith(b2n + ".")})
            self.fc3.load_state_dict({k[len(n3) + 1:]: v for k, v in sd.items()
                                      if k.startswith(n3 + ".")})

    # ------------------------------------------------- optimizer state in the full layout
    def _full_params(self):
        """[(full ToyMLP parameter name, this rank's parameter, layout)] in the full model's
        parameters() order; layout "rows" / "cols": this rank holds rows / columns
        [rank*s, (rank+1)*s) of the full tensor, "rep": the whole tensor (replicated)."""
        n1, n2, n3 = self._names
        b1n, b2n = self._bn_names
        out = [(f"{n1}.weight", self.fc1.weight, "rows")]
        if self.fc1.bias is not None:
            out.append((f"{n1}.bias", self.fc1.bias, "rows"))
        if self.bn1 is not None and self.bn1.weight is not None:
            out += [(f"{b1n}.weight", self.bn1.weight, "rows"),
                    (f"{b1n}.bias", self.bn1.bias, "rows")]
        out.append((f"{n2}.weight", self.fc2.weight, "cols"))
        if self.b2 is not None:
            out.append((f"{n2}.bias", self.b2, "rep"))
        if self.bn2 is not None and self.bn2.weight is not None:
            out += [(f"{b2n}.weight", self.bn2.weight, "rep"),
                    (f"{b2n}.bias", self.bn2.bias, "rep")]
        out += [(f"{n3}.{k}", q, "rep") for k, q in self.fc3.named_parameters()]
        return out

    def full_optim_state_dict(self, optimizer) -> dict:
        """``optimizer.state_dict()`` in the layout of an optimizer over the FULL ToyMLP's
        ``parameters()`` (collective: every rank must call it): each sharded state tensor
        (momentum, Adam's moments) is all-gathered from the ranks' slices the way
        ``full_state_dict`` gathers the weights, so a resumed job -- sharded at any W, or a DDP
        job -- gets the whole state, not rank 0's shard."""
        if len(optimizer.param_groups) != 1:
            raise ValueError("full_optim_state_dict: one parameter group over parameters()")
        local = optimizer.state_dict()
        order = optimizer.param_groups[0]["params"]
        pos = {id(q): i for i, q in enumerate(order)}
        full_state = {}
        for j, (_, q, how) in enumerate(self._full_params()):
            st = local["state"].get(pos[id(q)])
            # the same parameters have state on every rank (one group, same steps)
            if st is None:
                continue
            ent = {}
            for k, v in st.items():
                if not torch.is_tensor(v) or v.shape != q.shape or how == "rep":
                    ent[k] = v.detach().clone() if torch.is_tensor(v) else v
                elif how == "rows":
                    ent[k] = self._gather_rows(v)
                else:
                    ent[k] = self._gather_rows(v.t().contiguous()).t().contiguous()
            full_state[j] = ent
        group = {k: v for k, v in local["param_groups"][0].items() if k != "params"}
        group["params"] = list(range(len(self._full_params())))
        return {"state": full_state, "param_groups": [group]}

    def load_full_optim_state_dict(self, optimizer, sd: dict) -> None:
        """Inverse of ``full_optim_state_dict``: this rank keeps its slices of every sharded
        state tensor and loads them into ``optimizer`` (over this wrapper's parameters())."""
        if len(optimizer.param_groups) != 1 or len(sd["param_groups"]) != 1:
            raise ValueError("load_full_optim_state_dict: one parameter group")
        s = self._dims[1] // self.world
        lo, hi = self.rank * s, (self.rank + 1) * s
        order = optimizer.param_groups[0]["params"]
        pos = {id(q): i for i, q in enumerate(order)}
        state = {}
        for j, (name, q, how) in enumerate(self._full_params()):
            st = sd["state"].get(j)
            if st is None:
                continue
            ent = {}
            for k, v in st.items():
                if torch.is_tensor(v) and how != "rep" and v.dim() == q.dim() and \
                        v.numel() == q.numel() * self.world:
                    v = v[lo:hi] if how == "rows" else v[:, lo:hi]
                ent[k] = v.detach().clone().to(q.device) if torch.is_tensor(v) and v.dim() \
                    else v
                if torch.is_tensor(v) and v.dim() and ent[k].shape != q.shape:
                    raise ValueError(f"load_full_optim_state_dict: {name}.{k} has shape "
                                     f"{tuple(v.shape)}, this rank's slice needs "
                                     f"{tuple(q.shape)}")
            state[pos[id(q)]] = ent
        group = dict(sd["param_groups"][0])
        group["params"] = list(range(len(order)))
        self._fstate = None
        optimizer.load_state_dict({"state": state, "param_groups": [group]})


def rank_compute_ms(W: int, dims=(9216, 4096, 4096), classes: int = 10, B: int = 128,
                    steps: int = 100, optim: str = "sgd", device=None, fused: bool = True) -> float:
    """Measured per-rank compute of the W-rank tensor-sharded step on THIS one GPU: rank 0's
    shard shapes, every collective replaced by its local copy (set_fake_world), the node's batch
    gathered from a device dataset each step, SGD momentum (in the shards' GEMM epilogues unless
    ``fused=False``; or Adam), captured and replayed as bench.py runs it. The W-rank step is this plus its exposed collectives
    (parallel/commmodel.py simulate_tensor). World size 1 only (no process group peers)."""
    import time

    from .. import optim as toptim
    from .. import ops
    from ..data.synthetic import gather_batch
    from ..models import ToyMLP
    from ..train.graph import CapturedStep

    if runtime.get_world_size() != 1:
        raise RuntimeError("rank_compute_ms: a one-process measurement")
    dev = device or runtime.device()
    set_fake_world(W)
    try:
        torch.manual_seed(0)
        net = TensorParallelMLP(ToyMLP(in_features=dims[0], hidden=dims[1:],
                                       num_classes=classes, device=dev), global_batch=True)
        opt = toptim.SGD(net.parameters(), lr=0.01, momentum=0.9) if optim == "sgd" else \
            toptim.Adam(net.parameters(), lr=1e-3)
        if fused:
            net.register_fused_optimizer(opt)  # as bench.py runs it (SGD only)
        n = max(4 * W * B, 1024)
        data = torch.randn(n, dims[0], device=dev)
        labels = torch.randint(0, classes, (n,), device=dev)
        idx = torch.randperm(n, device=dev)[:W * B]

        def step():
            opt.zero_grad(set_to_none=True)
            x, y = gather_batch(data, labels, idx)
            ops.backward(ops.cross_entropy(net(x), y[:B]))
            net.sync_grads()
            opt.step()
        g = CapturedStep(step, warmup=3)
        for _ in range(10):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            g.replay()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1000.0 / steps
    finally:
        set_fake_world(0)
