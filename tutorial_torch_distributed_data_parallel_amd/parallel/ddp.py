"""DistributedDataParallel on the flat gradient arena + native reducer.

API-compatible with the way the reference uses torch DDP (``DDP(model, device_ids=[rank])``,
REF/multi-GPU-training-torch.py:245; Accelerate's ``prepare_model``, ACC/accelerator.py:1882-1896)
and with the rest of torch's constructor surface (bucket_cap_mb, broadcast_buffers,
find_unused_parameters, no_sync, state_dict with ``module.`` prefix, register_comm_hook for
gradient compression). Behaviour matched (SURVEY.md §4.3 oracles):
  1. after construction every rank holds rank 0's parameters and buffers (one broadcast of the
     flat arena, M3; buffers re-broadcast each forward when broadcast_buffers, M6);
  2. after backward ``param.grad == mean over ranks of the local gradients`` (ncclAvg);
  3. inside ``no_sync()`` gradients stay local and accumulate;
  4. parameter shapes are verified across ranks at construction (M2).
What differs by design (MI355X-first): gradients are bucket views from the start (no copies),
buckets follow backward order from iteration 0 (no 217 MiB first-iteration bucket, no rebuild),
a bucket may split a large tensor, all-reduces run on a dedicated high-priority HIP stream.
"""
from __future__ import annotations

import os

import contextlib
import hashlib
import weakref

import torch
import torch.distributed as dist
import torch.nn as nn

from .._native import native
from . import runtime as rt
from .arena import BufferArena, flatten_module

_MB = 1024 * 1024


def _param_signature(params) -> str:
    h = hashlib.sha1()
    for p in params:
        h.update(f"{tuple(p.shape)}:{p.dtype};".encode())
    return h.hexdigest()


def _verify_param_shapes(params):
    if rt.get_world_size() == 1:
        return
    sig = _param_signature(params)
    sigs = [None] * rt.get_world_size()
    dist.all_gather_object(sigs, (len(params), sig))
    if any(s != sigs[0] for s in sigs):
        raise RuntimeError(
            "DDP expects the same model on every rank: parameter count/shape/dtype signatures "
            f"differ across ranks: {sigs}")


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, device_ids=None, output_device=None, dim: int = 0,
                 broadcast_buffers: bool = True, process_group=None,
                 bucket_cap_mb: float | None = None, find_unused_parameters: bool = False,
                 check_reduction: bool = False, gradient_as_bucket_view: bool = True,
                 static_graph: bool = False, first_bucket_cap_mb: float | None = None,
                 split_bucket_mb: float | None = None, grad_compression: str | None = None,
                 timing: bool = False, check_replicas_every: int | None = None):
        super().__init__()
        if process_group is not None:
            raise NotImplementedError("sub-groups are not supported: DDP uses the world group")
        if not rt.is_initialized():
            raise RuntimeError("call init_process_group() before wrapping a model in DDP")
        self.module = module
        self.device_ids = device_ids
        self.output_device = output_device
        self.dim = dim
        self.broadcast_buffers = broadcast_buffers
        self.find_unused_parameters = find_unused_parameters
        self.static_graph = static_graph
        self.gradient_as_bucket_view = True  # always: gradients live in the bucket arena
        self.require_backward_grad_sync = True
        self.world_size = rt.get_world_size()
        self.rank = rt.get_rank()

        params = [p for p in module.parameters() if p.requires_grad]
        if not params:
            raise RuntimeError("DDP: module has no parameter that requires grad")
        devs = {p.device for p in params}
        if len(devs) != 1:
            raise ValueError(f"DDP expects all parameters on one device, got {devs}")
        self.device = next(iter(devs))
        if self.device.type == "cuda" and device_ids:
            want = torch.device("cuda", device_ids[0]) if isinstance(device_ids[0], int) \
                else torch.device(device_ids[0])
            if want != self.device:
                raise ValueError(f"module is on {self.device} but device_ids={device_ids}")
        self._gpu = self.device.type == "cuda"

        _verify_param_shapes(params)
        self.arena = flatten_module(module)
        self.buffers_arena = BufferArena(module)
        # M3: every rank starts from rank 0's weights -- one broadcast of the flat arena
        with torch.no_grad():
            rt.broadcast(self.arena.data, 0)
            self._sync_buffers()

        cap = (bucket_cap_mb if bucket_cap_mb is not None else 25.0) * _MB
        first = (first_bucket_cap_mb if first_bucket_cap_mb is not None else 1.0) * _MB
        split = (split_bucket_mb or 0.0) * _MB
        C = native() if self._gpu else None
        esize = self.arena.data.element_size()
        if C is not None:
            bounds = C.Reducer.compute_bucket_bounds(self.arena.offsets, self.arena.numels,
                                                     self.arena.numel, esize, int(first),
                                                     int(cap), int(split))
        else:
            bounds = _bucket_bounds_py(self.arena.offsets, self.arena.numels, self.arena.numel,
                                       esize, int(first), int(cap), int(split))
        self._bounds = bounds
        self._compression = grad_compression
        self._timing = timing
        self._build_reducer()
        self._hooks = []
        for i, p in enumerate(self.arena.params):
            self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))
        self._callback_queued = False
        self._iter = 0
        self._fused_opt = None
        self._epi_on = False
        self._epi_index = {}
        # SURVEY.md §5.2 debug mode: every N forwards, verify that all replicas hold bit-identical
        # parameters (a checksum all-gather); TDP_CHECK_REPLICAS=N sets it from the environment
        env_every = int(os.environ.get("TDP_CHECK_REPLICAS", "0") or 0)
        self.check_replicas_every = check_replicas_every if check_replicas_every is not None \
            else env_every

    # --------------------------------------------------------------------------- reducer
    def _build_reducer(self):
        nb = len(self._bounds) - 1
        if self._gpu:
            C = native()
            comp = {None: 0, "none": 0, "fp32": 0, "bf16": 1}[self._compression]
            comm = rt.comm()
            if comm is None:
                raise RuntimeError("GPU DDP needs the RCCL backend (init_process_group('nccl'))")
            # TDP_FORCE_COLLECTIVE=1 keeps the all-reduce (and its stream hop) at world size 1:
            # the single-GPU rehearsal of the multi-GPU schedule
            skip = os.environ.get("TDP_FORCE_COLLECTIVE", "0") != "1"
            self._backend = C.RcclBackend(comm, self.arena.grad, nb, compression=comp,
                                          timing=self._timing, skip_single_rank=skip)
            self.reducer = C.Reducer(self.arena.offsets, self.arena.numels, self._bounds,
                                     self._backend)
        else:
            self._works = []
            self._backend = None
            self.reducer = _make_py_reducer(self)

    def _make_hook(self, idx):
        arena = self.arena

        def hook(p):
            if not arena.is_arena_grad(idx):
                # a gradient produced outside the native ops: move it into its bucket slot
                slot = arena.grad_view(idx)
                slot.copy_(p.grad)
                p.grad = slot
            if self.require_backward_grad_sync and self.reducer.expecting:
                if not self._callback_queued:
                    torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
                    self._callback_queued = True
                self.reducer.mark_ready(idx, self._gpu)
        return hook

    def _finalize(self):
        self._callback_queued = False
        self.reducer.finalize(self._gpu, self.find_unused_parameters)
        self._iter += 1

    def _sync_buffers(self):
        if self.world_size == 1:
            return
        for flat in self.buffers_arena.flats:
            rt.broadcast(flat, 0)

    # --------------------------------------------------------------------------- debug
    def replica_checksum(self) -> torch.Tensor:
        """Bit-exact checksum of the flat parameter arena: [sum of the int32 words, sum of the
        words weighted by (index mod 65521) + 1] as int64 (order-sensitive, dtype-agnostic)."""
        with torch.no_grad():
            words = self.arena.data.view(torch.int32).to(torch.int64)
            w = (torch.arange(words.numel(), device=words.device, dtype=torch.int64) % 65521) + 1
            return torch.stack([words.sum(), (words * w).sum()])

    def check_replicas(self) -> None:
        """Raise if any rank's parameters differ from rank 0's (all-gather of the checksums)."""
        local = self.replica_checksum()
        if self.world_size == 1:
            return
        gathered = rt.all_gather_flat(local).view(self.world_size, 2)
        bad = [r for r in range(self.world_size) if not torch.equal(gathered[r], gathered[0])]
        if bad:
            raise RuntimeError(f"DDP replicas diverged at iteration {self._iter}: ranks {bad} "
                               f"hold different parameters than rank 0 "
                               f"(checksums {gathered.tolist()})")

    # --------------------------------------------------------------------------- nn.Module
    def forward(self, *inputs, **kwargs):
        if self.check_replicas_every and self._iter and \
                self._iter % self.check_replicas_every == 0 and torch.is_grad_enabled():
            self.check_replicas()
        if torch.is_grad_enabled() and self.require_backward_grad_sync:
            self.reducer.prepare_for_backward()
            if self._fused_opt is not None:
                # hyper-parameters as they are NOW (after any LR-scheduler step) drive this
                # iteration's in-reduction update
                self.push_fused_hyper(self._fused_opt)
        if self.broadcast_buffers and self.world_size > 1 and self.module.training:
            with torch.no_grad():
                self._sync_buffers()
        return self.module(*inputs, **kwargs)

    @contextlib.contextmanager
    def no_sync(self):
        old = self.require_backward_grad_sync
        self.require_backward_grad_sync = False
        try:
            yield
        finally:
            self.require_backward_grad_sync = old

    # --------------------------------------------------------------------------- fused optimizer
    def register_fused_optimizer(self, optimizer, shard: bool | None = None) -> bool:
        """Apply ``optimizer`` bucket by bucket inside the reduction (torch's
        ``DDP._register_fused_optim``): each bucket's parameters are updated right after its
        gradient is averaged. ``optimizer.step()`` becomes a no-op; the DDP forward hands the
        current hyper-parameters to the update. Requires a tdp SGD/Adam over exactly this DDP's
        parameters (one param group). Returns False (optimizer left unfused) on CPU.

        ``shard`` (default: world_size > 1) turns each bucket's all-reduce into reduce-scatter ->
        update of this rank's 1/W slice -> all-gather of the updated parameters (ZeRO stage 1
        inside DDP, cf. torch's ZeroRedundancyOptimizer): the same bytes over xGMI, 1/W of the
        optimizer's HBM traffic, identical parameters on every rank. Gradients are not averaged
        outside the owned slice afterwards, and optimizer state is only current in the owned
        slices until :meth:`consolidate_optimizer_state` (called by the checkpoint helpers).
        """
        from ..optim.fused import SGD, Adam

        if not self._gpu:
            return False
        if self.find_unused_parameters:
            raise ValueError("a fused optimizer needs every parameter to get a gradient")
        if len(optimizer.param_groups) != 1:
            raise ValueError("fused optimizer: exactly one parameter group is supported")
        params = optimizer.param_groups[0]["params"]
        if {id(p) for p in params} != {id(p) for p in self.arena.params}:
            raise ValueError("fused optimizer must own exactly the DDP model's parameters")
        if not isinstance(optimizer, (SGD, Adam)):
            raise TypeError("fused optimizer must be tdp.optim.SGD / Adam / AdamW")
        self._fused_opt = optimizer
        optimizer._fused_ddp = self
        self.push_fused_hyper(optimizer, initial=True)
        self._fused_shard = bool(self.world_size > 1 if shard is None else shard) and \
            self.world_size > 1
        self._backend.fused_shard = self._fused_shard
        # world size 1: the local gradient is already the average, so weight-gradient GEMMs may
        # apply the update in their epilogue (TDP_OPT_EPILOGUE=0 keeps the per-bucket update)
        self._epi_index = {id(p): i for i, p in enumerate(self.arena.params)}
        self._epi_on = (os.environ.get("TDP_OPT_EPILOGUE", "1") != "0" and
                        bool(self._backend.epilogue_allowed))
        if self._epi_on:
            me = weakref.ref(self)
            for p in self.arena.params:
                p._tdp_epi = me
        return True

    def epilogue_slot(self, p):
        """(backend, arena offset) for an optimizer-epilogue weight-gradient GEMM of ``p`` in the
        current backward, or None when the update must stay in the bucket path."""
        if not (self._epi_on and self.require_backward_grad_sync and self.reducer.expecting and
                self._backend.epilogue_allowed):
            return None
        i = self._epi_index.get(id(p))
        if i is None or not self.arena.numels[i]:
            return None
        return self._backend, self.arena.offsets[i]

    def consolidate_optimizer_state(self) -> None:
        """Make every rank's fused-optimizer state complete after sharded updates: all-gather
        each bucket's state slices in place (the tails are already replicated)."""
        if not getattr(self, "_fused_shard", False) or self._fused_opt is None:
            return
        opt = self._fused_opt
        bufs = opt._flat_bufs.get(id(self.arena), {})
        comm = rt.comm()
        W, r = self.world_size, self.rank
        for name, buf in bufs.items():
            if not torch.is_tensor(buf) or buf.numel() != self.arena.numel:
                continue
            for i in range(len(self._bounds) - 1):
                begin, end = self._bounds[i], self._bounds[i + 1]
                cnt = (end - begin) // W
                if cnt > 0:
                    comm.all_gather(buf[begin: begin + cnt * W],
                                    buf[begin + r * cnt: begin + (r + 1) * cnt])

    def push_fused_hyper(self, opt, initial: bool = False):
        from ..optim.fused import SGD

        g = opt.param_groups[0]
        a = self.arena
        if isinstance(opt, SGD):
            buf, fresh = None, False
            if g["momentum"] != 0:
                # fresh == the momentum buffers were just created: each bucket's first update
                # initialises them with the gradient (torch: buf = clone(grad))
                bufs, fresh = opt._flat_state(a, ("momentum_buffer",))
                buf = bufs["momentum_buffer"]
            self._backend.set_fused_sgd(a.data, buf, g["lr"], g["momentum"], g["dampening"],
                                        g["weight_decay"], g["nesterov"], g["maximize"],
                                        bool(fresh) and initial)
        else:
            keys = opt._keys(g)
            bufs, _ = opt._flat_state(a, keys)
            step = opt._current_flat_step(a) if initial else self._backend.fused_adam_step
            b1, b2 = g["betas"]
            self._backend.set_fused_adam(a.data, bufs["exp_avg"], bufs["exp_avg_sq"],
                                         bufs.get("max_exp_avg_sq"), g["lr"], b1, b2, g["eps"],
                                         g["weight_decay"], g["amsgrad"], g["maximize"],
                                         opt._decoupled, int(step))

    def register_comm_hook(self, state, hook):
        """Gradient compression hooks: torch's bf16_compress_hook (or the string "bf16")."""
        name = hook if isinstance(hook, str) else getattr(hook, "__name__", "")
        if name in ("bf16", "bf16_compress_hook"):
            self._compression = "bf16"
        elif name in ("allreduce_hook", "none", "fp32"):
            self._compression = None
        else:
            raise NotImplementedError(f"comm hook {name!r} is not supported (bf16 | fp32)")
        if self._gpu:
            self._build_reducer()
            if self._fused_opt is not None:
                self.push_fused_hyper(self._fused_opt, initial=False)

    # --------------------------------------------------------------------------- logging
    def _get_ddp_logging_data(self) -> dict:
        b = self._bounds
        esize = self.arena.data.element_size()
        return {
            "world_size": self.world_size,
            "backend_name": rt.get_backend(),
            "bucket_cap_bytes": None,
            "bucket_sizes": [(b[i + 1] - b[i]) * esize for i in range(len(b) - 1)],
            "num_buckets": len(b) - 1,
            "has_rebuilt_buckets": 0,
            "iterations": self._iter,
            "gradient_as_bucket_view": True,
            "find_unused_parameters": self.find_unused_parameters,
            "first_iteration_ready_order": list(self.reducer.ready_order()),
            "avg_backward_comm_time_ms": self.reducer.last_comm_ms(),
            "grad_compression": self._compression or "none",
        }


def _bucket_bounds_py(offsets, numels, arena_numel, esize, first_cap, cap, split):
    """Python twin of Reducer::compute_bucket_bounds (used when no native module: CPU)."""
    b = [0]
    cur = 0
    split_el = max(split // esize, 1) if split > 0 else 0
    for i, (o, n) in enumerate(zip(offsets, numels)):
        c = first_cap if len(b) == 1 else cap
        nbytes = n * esize
        if cur > 0 and cur + nbytes > c:
            b.append(o)
            cur = 0
        if split_el and n > split_el:
            if b[-1] != o:
                b.append(o)
            b.extend(o + s for s in range(split_el, n, split_el))
            if i + 1 < len(offsets):
                b.append(o + n)
            cur = 0
            continue
        cur += nbytes
    if b[-1] != arena_numel:
        b.append(arena_numel)
    out = [b[0]]
    for x in b[1:]:
        if x > out[-1]:
            out.append(x)
    if len(out) == 1:
        out.append(arena_numel)
    return out


def _make_py_reducer(ddp: DistributedDataParallel):
    """Reducer over torch.distributed (gloo) for CPU runs. Uses the native C++ Reducer logic
    when the extension is importable (it is, on every supported machine), else a Python twin."""
    arena = ddp.arena
    world = ddp.world_size

    def launch(bucket, begin, end):
        t = arena.grad[begin:end]
        if world > 1:
            t.div_(world)  # DDP semantics: divide, then SUM (gloo has no AVG)
            ddp._works.append(dist.all_reduce(t, async_op=True))

    def wait():
        for w in ddp._works:
            w.wait()
        ddp._works.clear()

    def zero(begin, end):
        arena.grad[begin:end].zero_()

    try:
        C = native()
        backend = C.PyBackend(launch, wait, zero)
        return C.Reducer(arena.offsets, arena.numels, ddp._bounds, backend)
    except Exception:  # pragma: no cover - extension missing on a CPU-only box
        return _PyReducer(arena.offsets, arena.numels, ddp._bounds, launch, wait, zero)


class _PyReducer:
    def __init__(self, offsets, numels, bounds, launch, wait, zero):
        self.offsets, self.numels, self.bounds = offsets, numels, bounds
        self._launch, self._wait, self._zero = launch, wait, zero
        nb = len(bounds) - 1
        self.param_buckets = []
        self.nparams = [0] * nb
        for o, n in zip(offsets, numels):
            bs = [b for b in range(nb) if n and bounds[b] < o + n and bounds[b + 1] > o]
            self.param_buckets.append(bs)
            for b in bs:
                self.nparams[b] += 1
        self.expecting = False
        self.iteration = 0
        self.num_buckets = nb
        self._order = []

    def prepare_for_backward(self):
        self.pending = list(self.nparams)
        self.ready = [n == 0 for n in self.nparams]
        self.pready = [False] * len(self.offsets)
        self.next = 0
        self.expecting = True

    def mark_ready(self, p, gpu=False):
        if not self.expecting:
            return
        if self.pready[p]:
            raise RuntimeError("Expected to mark a variable ready only once")
        self.pready[p] = True
        if self.iteration == 0:
            self._order.append(p)
        for b in self.param_buckets[p]:
            self.pending[b] -= 1
            if self.pending[b] == 0:
                self.ready[b] = True
        self._launch_ready()

    def _launch_ready(self):
        while self.next < self.num_buckets and self.ready[self.next]:
            self._launch(self.next, self.bounds[self.next], self.bounds[self.next + 1])
            self.next += 1

    def finalize(self, gpu=False, allow_unused=False):
        if not self.expecting:
            return
        unready = [i for i, r in enumerate(self.pready) if not r and self.numels[i]]
        if unready and not allow_unused:
            raise RuntimeError(f"parameters {unready} received no gradient; pass "
                               "find_unused_parameters=True")
        for p in unready:
            self._zero(self.offsets[p], self.offsets[p] + self.numels[p])
            self.pready[p] = True
            for b in self.param_buckets[p]:
                self.pending[b] -= 1
                if self.pending[b] == 0:
                    self.ready[b] = True
        self._launch_ready()
        self._wait()
        self.expecting = False
        self.iteration += 1

    def bucket_bounds(self):
        return list(self.bounds)

    def ready_order(self):
        return list(self._order)

    def last_comm_ms(self):
        return -1.0


DDP = DistributedDataParallel
