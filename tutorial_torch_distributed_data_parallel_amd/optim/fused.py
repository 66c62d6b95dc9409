"""Fused SGD / Adam / AdamW (torch.optim-compatible).

The reference steps ``torch.optim.Adam(ddp_model.parameters(), lr=0.001)``
(REF/multi-GPU-training-torch.py:249, REF/multi-GPU-training-accelerate.py:126); the north star
adds a fused SGD. Both are ``torch.optim.Optimizer`` subclasses (param_groups, state_dict,
load_state_dict, LR schedulers all work) whose ``step`` is:
  * FLAT  -- when the group's parameters are exactly one ParamArena (every DDP model, or any model
             passed through ``flatten_module``) and each .grad is its arena view: ONE kernel over
             the whole arena, optimizer state kept in arena-shaped flat buffers
             (state[p][...] are views into them);
  * MULTI -- otherwise: one launch over a device-side chunk table of the individual tensors;
  * CPU   -- torch's own single-tensor implementation (reference path for the CPU tests).
Semantics are torch's (TORCH/optim/sgd.py, TORCH/optim/adam.py): momentum buffer initialised to
the first gradient, dampening, nesterov, maximize, L2 vs decoupled weight decay, amsgrad,
bias-corrected Adam with a per-parameter step counter.
"""
from __future__ import annotations

import functools
import weakref

import torch
from torch.optim import Optimizer
from torch.optim.optimizer import _global_optimizer_post_hooks, _global_optimizer_pre_hooks

from .._native import native
from ..parallel.arena import arena_of


def _flat_arena(group):
    params = group["params"]
    a = arena_of(params)
    if a is None:
        return None
    for i in range(len(a.params)):
        if not a.is_arena_grad(i):
            return None
    return a


def _hooks_or_profiler(opt) -> bool:
    return bool(_global_optimizer_pre_hooks or _global_optimizer_post_hooks or
                opt._optimizer_step_pre_hooks or opt._optimizer_step_post_hooks or
                torch.autograd.profiler._is_profiler_enabled)


def _lean_step_hook(func):
    """torch wraps ``step`` (TORCH/optim/optimizer.py ``profile_hook_step``) in a record_function
    range plus the hook dispatch on EVERY call: ~10 us of host time per training step, and the
    eager toy-MLP step is host-bound right after the loss (profiles/host_overhead.md). Same
    behaviour, paid only when a hook is registered or the profiler is on."""

    @functools.wraps(func)
    def wrapper(self, *args, **kwargs):
        if _hooks_or_profiler(self):
            return Optimizer.profile_hook_step(func)(self, *args, **kwargs)
        out = func(self, *args, **kwargs)
        self._optimizer_step_code()
        return out

    wrapper.hooked = True  # torch's _patch_step_function leaves a hooked step alone
    return wrapper


_LIVE = weakref.WeakSet()  # optimizers that own device hyper blocks (CapturedStep re-syncs them)


def hyper_slots() -> dict:
    """Slot indices of the device hyper block (csrc/kernels.h HyperSlot)."""
    global _SLOTS
    if _SLOTS is None:
        _SLOTS = dict(native().hyper_slots())
    return _SLOTS


_SLOTS = None


def sync_all_hyper() -> None:
    """Push host-side hyper-parameter changes (LR schedulers, ...) of every live optimizer into
    its device hyper block; called before each hipGraph replay (train/graph.py)."""
    for opt in list(_LIVE):
        opt.sync_hyper()



def _dense(t: torch.Tensor) -> torch.Tensor:
    """A 1-D view of ``t``'s memory in storage order (no copy): the elementwise optimizer kernels
    only need p, grad and state to share one element order. Dense row-major tensors and
    channels_last conv weights (the native convolutions' parameter layout) qualify."""
    if t.is_contiguous():
        return t.view(-1)
    if t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last):
        return t.permute(0, 2, 3, 1).view(-1)
    raise RuntimeError(f"optimizer tensor with unsupported strides {tuple(t.stride())}")


def _grad_like(p: torch.Tensor) -> torch.Tensor:
    """``p.grad`` flattened in ``p``'s element order (converted only if its layout differs)."""
    g = p.grad
    if p.is_contiguous():
        return g.contiguous().view(-1)
    return _dense(g.contiguous(memory_format=torch.channels_last))

class _FusedBase(Optimizer):
    _state_keys: tuple = ()
    _kind = 0  # hyper-block kind: 1 SGD, 2 Adam

    def __init__(self, params, defaults):
        super().__init__(params, defaults)
        self._flat_bufs = {}  # id(arena) -> {key: flat tensor}
        self._flat_step = {}  # id(arena) -> int step shared by every arena parameter (Adam)
        self._blocks = {}     # group index -> [device hyper block, host copy of its scalars]

    def __init_subclass__(cls, **kwargs):
        super().__init_subclass__(**kwargs)
        if "step" in cls.__dict__ and not getattr(cls.__dict__["step"], "hooked", False):
            cls.step = _lean_step_hook(cls.__dict__["step"])

    # ------------------------------------------------------------------ device hyper block
    def _scalars(self, g) -> tuple:
        raise NotImplementedError

    def hyper_block(self, gi: int = 0, device=None, step: int = 0,
                    first: bool = False) -> torch.Tensor:
        """The device-resident hyper-parameter block of parameter group ``gi`` (created on first
        use with step count ``step``; ``first`` = the next step initialises the SGD momentum
        buffers). Kernels read lr / momentum / betas / bias corrections from it, so a captured
        hipGraph replays with the current values (csrc/kernels.h HyperSlot)."""
        ent = self._blocks.get(gi)
        if ent is not None:
            return ent[0]
        S = hyper_slots()
        g = self.param_groups[gi]
        dev = device if device is not None else g["params"][0].device
        vals = self._scalars(g)
        host = torch.zeros(S["size"], dtype=torch.float32)
        host[:len(vals)] = torch.tensor(vals, dtype=torch.float64).float()
        host[S["scale"]] = 1.0
        host[S["first_next"]] = 1.0 if first else 0.0
        host.view(torch.int32)[S["step"]] = int(step)
        blk = host.to(dev)
        self._blocks[gi] = [blk, vals]
        _LIVE.add(self)
        return blk

    def sync_hyper(self) -> None:
        """Stream-ordered write of changed scalars (lr, momentum / betas, weight decay, eps) into
        the device blocks. Nothing is issued when nothing changed."""
        for gi, ent in self._blocks.items():
            vals = self._scalars(self.param_groups[gi])
            if vals == ent[1]:
                continue
            blk = ent[0]
            if blk.is_cuda and torch.cuda.is_current_stream_capturing():
                raise RuntimeError("hyper-parameters changed while a hipGraph was being captured")
            src = torch.tensor(vals, dtype=torch.float64).float()
            if blk.is_cuda:
                blk[:len(vals)].copy_(src.pin_memory(), non_blocking=True)
            else:
                blk[:len(vals)].copy_(src)
            ent[1] = vals

    def device_step(self, gi: int = 0):
        """Step count held by the device block of group ``gi`` (None without a block). Reading
        it synchronises with the device."""
        ent = self._blocks.get(gi)
        if ent is None:
            return None
        return int(ent[0].view(torch.int32)[hyper_slots()["step"]].item())

    def _request_first(self, blk) -> None:
        blk[hyper_slots()["first_next"]] = 1.0

    # ------------------------------------------------------------------ torch API
    def zero_grad(self, set_to_none: bool = True) -> None:
        """torch's zero_grad, without its per-call record_function range / dynamo guard when
        gradients are simply dropped (the default) and the profiler is off."""
        if not set_to_none or torch.autograd.profiler._is_profiler_enabled:
            return super().zero_grad(set_to_none)
        for g in self.param_groups:
            for p in g["params"]:
                p.grad = None

    def _flat_state(self, arena, keys):
        """Arena-shaped state buffers; adopts values already in self.state (load_state_dict)."""
        bufs = self._flat_bufs.get(id(arena))
        if bufs is not None and all(k in bufs for k in keys):
            return bufs, False  # steady state: no per-parameter Python work
        fresh = False
        if bufs is None:
            bufs = {k: arena.new_state() for k in keys}
            self._flat_bufs[id(arena)] = bufs
            fresh = True
            if not hasattr(arena, "_optimizers"):
                arena._optimizers = weakref.WeakSet()
            arena._optimizers.add(self)  # a DDP bucket rebuild re-lays the state out too
        for i, p in enumerate(arena.params):
            st = self.state[p]
            for k in keys:
                view = arena.state_view(bufs[k], i)
                cur = st.get(k)
                if cur is None:
                    st[k] = view
                elif cur.data_ptr() != view.data_ptr():
                    view.copy_(cur)
                    st[k] = view
                    fresh = False
        return bufs, fresh

    def _relayout(self, arena, remap) -> None:
        """The arena was re-laid out (DDP bucket rebuild): move the flat state buffers the same
        way and re-point the per-parameter state views."""
        bufs = self._flat_bufs.get(id(arena))
        if not bufs:
            return
        for k in list(bufs):
            bufs[k] = remap(bufs[k])
        for i, p in enumerate(arena.params):
            st = self.state[p]
            for k, buf in bufs.items():
                st[k] = arena.state_view(buf, i)

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._flat_bufs = {}  # re-adopted into flat buffers on the next step
        self._flat_step = {}
        self._blocks = {}     # re-created with the loaded step count
        ddp = getattr(self, "_fused_ddp", None)
        if ddp is not None:
            ddp.push_fused_hyper(self, initial=True)

    def _fused_step(self) -> bool:
        """When a DDP model applies this optimizer inside its reduction the update already
        happened during backward, so step() has nothing left to do (the DDP forward hands the
        current hyper-parameters, e.g. after an LR-scheduler step, to the fused update)."""
        return getattr(self, "_fused_ddp", None) is not None

    def _current_flat_step(self, arena) -> int:
        if id(arena) in self._flat_step:
            return self._flat_step[id(arena)]
        steps = {int(self.state[p]["step"].item()) if torch.is_tensor(self.state[p].get("step"))
                 else int(self.state[p].get("step") or 0) for p in arena.params}
        return max(steps) if steps else 0

    def state_dict(self):
        # materialise the flat step counter (held by the device block: graph replays advance it
        # without the host) into torch's per-parameter "step" entries
        if self._kind == 2:
            for gi, g in enumerate(self.param_groups):
                a = arena_of(g["params"])
                dstep = self.device_step(gi)
                if a is not None and dstep is not None:
                    self._flat_step[id(a)] = dstep
        for g in self.param_groups:
            a = arena_of(g["params"])
            if a is not None and id(a) in self._flat_step:
                t = torch.tensor(float(self._flat_step[id(a)]))
                for p in a.params:
                    self.state[p]["step"] = t.clone()
        return super().state_dict()


class SGD(_FusedBase):
    def __init__(self, params, lr: float = 1e-3, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False, *, maximize: bool = False,
                 grad_scale: float = 1.0):
        if lr < 0 or momentum < 0 or weight_decay < 0:
            raise ValueError("invalid SGD hyper-parameter")
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=dampening,
                                      weight_decay=weight_decay, nesterov=nesterov,
                                      maximize=maximize, grad_scale=grad_scale))

    _kind = 1

    def _scalars(self, g) -> tuple:
        return (float(g["lr"]), float(g["momentum"]), float(g["dampening"]),
                float(g["weight_decay"]), 0.0)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if self._fused_step():
            return loss
        tp = getattr(self, "_fused_tp", None)
        tp = tp() if tp is not None else None
        if tp is not None:
            # tensor-sharded wrapper with the shards' update in their GEMM epilogues: the rest
            tp._fused_step(self)
            return loss
        for gi, g in enumerate(self.param_groups):
            ps = [p for p in g["params"] if p.grad is not None]
            if not ps:
                continue
            hyper = (g["lr"], g["momentum"], g["dampening"], g["weight_decay"], g["nesterov"],
                     g["maximize"])
            if not ps[0].is_cuda:
                self._cpu_step(g, ps)
                continue
            C = native()
            mom = g["momentum"] != 0
            arena = _flat_arena(g) if len(ps) == len(g["params"]) else None
            if arena is not None:
                buf, fresh = None, False
                if mom:
                    # fresh == the buffers were just created (torch: buf = clone(grad))
                    bufs, fresh = self._flat_state(arena, ("momentum_buffer",))
                    buf = bufs["momentum_buffer"]
                # scalars and the first-step flag come from the device block (graph-safe)
                if gi in self._blocks:
                    blk = self._blocks[gi][0]
                    self.sync_hyper()
                    if fresh:
                        self._request_first(blk)
                else:
                    blk = self.hyper_block(gi, first=fresh)
                C.opt_step_begin(blk, 1)
                C.sgd_flat(arena.data, arena.grad, buf, *hyper[:5], hyper[5], False,
                           g["grad_scale"], hyper=blk)
                continue
            new, old = [], []
            for p in ps:
                st = self.state[p]
                if mom and st.get("momentum_buffer") is None:
                    st["momentum_buffer"] = torch.empty_like(p)
                    new.append(p)
                else:
                    old.append(p)
            for lst, first in ((new, True), (old, False)):
                if lst:
                    bufs = [self.state[p]["momentum_buffer"] for p in lst] if mom else []
                    C.sgd_multi([_dense(p.data) for p in lst], [_grad_like(p) for p in lst],
                                [_dense(b) for b in bufs], *hyper[:5], hyper[5], first,
                                g["grad_scale"])
        return loss

    def _cpu_step(self, g, ps):
        for p in ps:
            d = p.grad * g["grad_scale"]
            if g["maximize"]:
                d = -d
            if g["weight_decay"]:
                d = d.add(p, alpha=g["weight_decay"])
            if g["momentum"]:
                st = self.state[p]
                buf = st.get("momentum_buffer")
                if buf is None:
                    buf = d.clone()
                    st["momentum_buffer"] = buf
                else:
                    buf.mul_(g["momentum"]).add_(d, alpha=1 - g["dampening"])
                d = d.add(buf, alpha=g["momentum"]) if g["nesterov"] else buf
            p.add_(d, alpha=-g["lr"])


class Adam(_FusedBase):
    _decoupled = False

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, amsgrad: bool = False, *, maximize: bool = False,
                 grad_scale: float = 1.0):
        if not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"invalid betas {betas}")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps,
                                      weight_decay=weight_decay, amsgrad=amsgrad,
                                      maximize=maximize, grad_scale=grad_scale))

    _kind = 2

    def _scalars(self, g) -> tuple:
        b1, b2 = g["betas"]
        return (float(g["lr"]), float(b1), float(b2), float(g["weight_decay"]), float(g["eps"]))

    def _keys(self, g):
        return ("exp_avg", "exp_avg_sq") + (("max_exp_avg_sq",) if g["amsgrad"] else ())

    def _bump_step(self, ps):
        steps = set()
        for p in ps:
            st = self.state[p]
            s = st.get("step")
            s = torch.tensor(0.0) if s is None else s
            s = s + 1 if torch.is_tensor(s) else torch.tensor(float(s) + 1)
            st["step"] = s
            steps.add(int(s.item()) if torch.is_tensor(s) else int(s))
        return steps

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if self._fused_step():
            return loss
        for gi, g in enumerate(self.param_groups):
            ps = [p for p in g["params"] if p.grad is not None]
            if not ps:
                continue
            b1, b2 = g["betas"]
            if not ps[0].is_cuda:
                self._cpu_step(g, ps)
                continue
            C = native()
            keys = self._keys(g)
            args = (g["lr"], b1, b2, g["eps"], g["weight_decay"], g["amsgrad"], g["maximize"],
                    self._decoupled)
            arena = _flat_arena(g) if len(ps) == len(g["params"]) else None
            if arena is not None:
                key = id(arena)
                if key not in self._flat_step:
                    prev = {int(self.state[p]["step"].item()) if torch.is_tensor(
                        self.state[p].get("step")) else int(self.state[p].get("step") or 0)
                        for p in arena.params}
                    if len(prev) == 1:
                        self._flat_step[key] = prev.pop()
                if key in self._flat_step:
                    bufs, _ = self._flat_state(arena, keys)
                    # the step count and bias corrections advance ON THE DEVICE (opt_step_begin),
                    # so a captured step replays correctly; the host count mirrors it eagerly
                    if gi in self._blocks:
                        blk = self._blocks[gi][0]
                        self.sync_hyper()
                    else:
                        blk = self.hyper_block(gi, step=self._flat_step[key])
                    self._flat_step[key] += 1
                    C.opt_step_begin(blk, 2)
                    C.adam_flat(arena.data, arena.grad, bufs["exp_avg"], bufs["exp_avg_sq"],
                                bufs.get("max_exp_avg_sq"), *args, self._flat_step[key],
                                g["grad_scale"], hyper=blk)
                    continue
            for k2 in list(self._flat_step):  # leaving the flat path: write the counter back
                a2 = arena_of(g["params"])
                if a2 is not None and id(a2) == k2:
                    dstep = self.device_step(gi)
                    self._blocks.pop(gi, None)
                    t = torch.tensor(float(dstep if dstep is not None else
                                           self._flat_step[k2]))
                    self._flat_step.pop(k2)
                    for p in a2.params:
                        self.state[p]["step"] = t.clone()
            by_step = {}
            for p in ps:
                st = self.state[p]
                for k in keys:
                    if st.get(k) is None:
                        st[k] = torch.zeros_like(p)
            self._bump_step(ps)
            for p in ps:
                by_step.setdefault(int(self.state[p]["step"].item()), []).append(p)
            for step, lst in by_step.items():
                st = [self.state[p] for p in lst]
                C.adam_multi([_dense(p.data) for p in lst], [_grad_like(p) for p in lst],
                             [_dense(s["exp_avg"]) for s in st], [_dense(s["exp_avg_sq"]) for s in st],
                             [_dense(s["max_exp_avg_sq"]) for s in st] if g["amsgrad"] else [],
                             *args, step, g["grad_scale"])
        return loss

    def _cpu_step(self, g, ps):
        b1, b2 = g["betas"]
        for p in ps:
            st = self.state[p]
            if st.get("exp_avg") is None:
                st["exp_avg"] = torch.zeros_like(p)
                st["exp_avg_sq"] = torch.zeros_like(p)
                if g["amsgrad"]:
                    st["max_exp_avg_sq"] = torch.zeros_like(p)
            self._bump_step([p])
            t = int(st["step"].item())
            grad = p.grad * g["grad_scale"]
            if g["maximize"]:
                grad = -grad
            if g["weight_decay"]:
                if self._decoupled:
                    p.mul_(1 - g["lr"] * g["weight_decay"])
                else:
                    grad = grad.add(p, alpha=g["weight_decay"])
            m, v = st["exp_avg"], st["exp_avg_sq"]
            m.lerp_(grad, 1 - b1)
            v.mul_(b2).addcmul_(grad, grad, value=1 - b2)
            bc1 = 1 - b1 ** t
            bc2s = (1 - b2 ** t) ** 0.5
            vv = v
            if g["amsgrad"]:
                torch.maximum(st["max_exp_avg_sq"], v, out=st["max_exp_avg_sq"])
                vv = st["max_exp_avg_sq"]
            denom = (vv.sqrt() / bc2s).add_(g["eps"])
            p.addcdiv_(m, denom, value=-g["lr"] / bc1)


class AdamW(Adam):
    _decoupled = True

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 1e-2, amsgrad: bool = False, *, maximize: bool = False,
                 grad_scale: float = 1.0):
        super().__init__(params, lr, betas, eps, weight_decay, amsgrad, maximize=maximize,
                         grad_scale=grad_scale)
