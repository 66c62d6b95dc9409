"""Whole-step HIP graph capture ("HIP graphs instead of a tracing compiler").

A data-parallel training step of the toy MLP is ~25 kernel launches plus autograd, DDP hooks and
optimizer bookkeeping in Python. ``CapturedStep`` records one complete step -- on-device batch
gather, forward, loss, backward with the reducer's bucketed RCCL all-reduces on the comm stream,
optimizer update -- into a hipGraph once, then each iteration is one graph launch.

When it pays (measured on MI355X, profiles/bench/mode*.json): the first eager implementation left
50-175 us host gaps between kernels and capture cut the step from 1.67 to 0.64 ms; after the
host path was trimmed (device-resident sampler indices, one flat optimizer kernel) the eager step
is GPU-bound (0.62 ms) and replay brings nothing on one GPU. Capture still matters for the
multi-GPU schedule: inside a graph the reducer's all-reduces run on a side stream and overlap
backward for free, whereas eagerly a cross-queue wait left pending while the host runs ahead
slows every kernel (the reducer therefore runs eager collectives on the compute stream).

Contract (as for torch.cuda.graphs): the captured function reads its varying inputs from static
tensors the caller refreshes before ``replay`` (here: a device index tensor for the batch);
optimizer state and gradients live in fixed buffers (the flat arenas), so replay updates them in
place. Per-step optimizer scalars are NOT baked in: every tdp optimizer keeps lr, momentum /
betas, weight decay, the Adam step count and bias corrections in a device hyper block
(csrc/kernels.h HyperSlot) that the kernels read; ``replay`` first pushes host-side changes
(an LR scheduler's step) into those blocks with stream-ordered copies, and the captured
``opt_step_begin`` kernel advances the step count on the device. Structural changes (momentum
switched on/off, amsgrad, a new parameter group) still need a re-capture. The ``warmup`` steps
really execute; the capturing call only records (it does not advance the model), so after
construction the model has taken exactly ``warmup`` steps.
"""
from __future__ import annotations

import os
import weakref

import torch


class CaptureFailed(RuntimeError):
    """The hipGraph capture itself failed (the warm-up steps ran fine)."""


def _capture_fault_injected() -> bool:
    """TDP_FAULT_CAPTURE=<rank>: make that rank's capture fail (the agreement tests)."""
    spec = os.environ.get("TDP_FAULT_CAPTURE")
    if not spec:
        return False
    from ..parallel import runtime as rt

    return int(spec) == rt.get_rank()


class CapturedStep:
    def __init__(self, step_fn, warmup: int = 3, pool=None):
        if not torch.cuda.is_available():
            raise RuntimeError("CapturedStep needs a GPU")
        from ..parallel.ddp import _LIVE

        self.step_fn = step_fn
        iter0 = {id(d): d._iter for d in list(_LIVE)}
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):  # allocator warm-up, lazy kernel attributes, momentum init
                step_fn()
        torch.cuda.current_stream().wait_stream(side)
        # a bucket rebuild planned by the warm-up must happen now, eagerly: recorded into the
        # graph, its relayout would restore the pre-capture buffers at every replay
        live = list(_LIVE)
        # the DDPs this step drives: those the warm-up advanced (without a warm-up: every live
        # one, the conservative answer)
        used = [d for d in live if warmup == 0 or d._iter != iter0.get(id(d), d._iter)]
        if any(d.find_unused_parameters for d in used):
            # which parameters went unused is decided on the host every iteration (the reducer
            # zeroes their slots): a graph would freeze the capture-time answer. The flag is a
            # constructor argument, identical on every rank, so every rank refuses alike -- and
            # BEFORE recording: a recorded-but-never-replayed step would have advanced the
            # reducer's, the optimizer's and the factored jobs' host-side state
            torch.cuda.synchronize()
            raise CaptureFailed("DDP(find_unused_parameters=True): the unused-parameter set is "
                                "host bookkeeping per iteration; the step runs eagerly")
        for d in live:
            d.settle()
        torch.cuda.synchronize()
        if _capture_fault_injected():
            raise CaptureFailed("injected capture fault (TDP_FAULT_CAPTURE)")
        # DDP's host-side per-iteration logic (its iteration counter, which drives
        # check_replicas_every) runs while the step is recorded but not on replays: note the
        # counters, restore them after the capture -- on success AND failure, so ranks that
        # captured and ranks that did not agree on the count -- and advance them per replay
        before = {id(d): (d, d._iter) for d in live}
        self.graph = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(self.graph, pool=pool):
                self.output = step_fn()
        except Exception as e:
            raise CaptureFailed(repr(e)) from e
        finally:
            self._ddps = []  # (DDP, iterations one replay runs: a graph may hold several steps)
            for d, it in before.values():
                if d._iter != it:
                    self._ddps.append((weakref.ref(d), d._iter - it))
                    d._iter = it
        torch.cuda.synchronize()

    def replay(self):
        from ..optim.fused import sync_all_hyper

        sync_all_hyper()  # LR schedules etc. reach the captured kernels through the hyper blocks
        self.graph.replay()
        from ..parallel import runtime as rt

        comm = rt.comm()
        if comm is not None and comm.world > 1:
            comm.watch_current("captured training step")  # RCCL watchdog covers the replay
        for ref, n in self._ddps:
            d = ref()
            if d is None:
                continue
            before = d._iter
            d._iter += n
            # the eager forward checks before the step whose count is a multiple: same cadence
            # (once per replay that crosses a multiple), run outside the graph (it is a
            # collective: every rank replays in lock-step)
            k = d.check_replicas_every
            if k and d._iter // k > before // k:
                d.check_replicas()
        return self.output

    __call__ = replay


def agree(ok: bool) -> bool:
    """True only if ``ok`` holds on EVERY rank (a 1-element MIN all-reduce over gloo on the host:
    independent of the GPU stream state a failed capture may leave behind)."""
    from ..parallel import runtime as rt

    if not rt.is_initialized() or rt.get_world_size() == 1:
        return ok
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    rt.all_reduce(t, "min")
    return bool(int(t[0]))


def _clear_capture_error() -> None:
    """Clear the thread's sticky HIP error a failed capture leaves (torch.cuda.graph's exit has
    ended the capture): otherwise the next checked launch of the EAGER fallback reports the
    capture's error (seen at W = 4 after a one-rank capture failure: the barrier that followed
    raised, the other ranks stalled)."""
    try:
        from .._native import native

        msg = native().take_last_hip_error()
    except Exception:  # noqa: BLE001 - an older build without the binding
        msg = ""
    if msg:
        import sys

        print(f"[tdp] cleared the failed capture's HIP error: {msg}", file=sys.stderr, flush=True)


def try_capture(step_fn, warmup: int = 3, log=print, capture=CapturedStep):
    """Capture if possible, else run eagerly -- decided for ALL ranks together: one rank
    replaying a graph while another runs eagerly would issue collectives in a different order
    (a deadlock or silent corruption). Warm-up errors propagate; a capture error on any rank
    makes every rank return the eager ``step_fn``. Returns the replayable step or ``step_fn``."""
    graph, err = None, None
    try:
        graph = capture(step_fn, warmup=warmup)
    except CaptureFailed as e:
        err = e
        if torch.cuda.is_available():
            _clear_capture_error()
            torch.cuda.synchronize()
    if agree(graph is not None):
        return graph
    if err is not None:
        log(f"[tdp] hipGraph capture failed, running eagerly on every rank: {err}")
    else:
        log("[tdp] hipGraph capture failed on another rank: running eagerly on every rank")
    del graph
    return step_fn


def _static_like(t: torch.Tensor) -> torch.Tensor:
    """An uninitialised buffer with ``t``'s shape, dtype and memory layout (a channel-padded
    channels_last batch keeps its padded base: the NHWC convolutions read that)."""
    base = getattr(t, "_tdp_padded_base", None)
    if base is not None:
        from ..data.synthetic import _padded_view

        return _padded_view(torch.empty_like(base), t.shape[1])
    return torch.empty_like(t)  # preserve_format: channels_last stays channels_last


def _layout(t: torch.Tensor):
    base = getattr(t, "_tdp_padded_base", None)
    return (tuple(t.shape), t.dtype, t.device, tuple(t.stride()),
            None if base is None else tuple(base.shape))


def _fill(dst: torch.Tensor, src: torch.Tensor) -> None:
    db, sb = getattr(dst, "_tdp_padded_base", None), getattr(src, "_tdp_padded_base", None)
    if db is not None and sb is not None:
        db.copy_(sb, non_blocking=True)
    else:
        dst.copy_(src, non_blocking=True)


class GraphedStep:
    """A training step ``body(x, y)`` replayed as a hipGraph fed by static input buffers.

    This is how the reference's own entry points (REF/multi-GPU-training-torch.py:104-133
    ``train``; REF/multi-GPU-training-accelerate.py:39-57) get their gradient all-reduce
    overlapped with backward, as stock DDP gives it to them: inside a captured step the
    reducer's bucket collectives run on the communicator's side stream behind graph edges
    (csrc/reducer.cpp pick_stream), whereas eagerly they run on the compute stream.

    The first ``warmup`` calls run ``body`` eagerly -- each on its own real batch, so training
    is step-for-step the eager computation: these steps agree the factored-sync slot sizes,
    trigger the one-time bucket rebuild and initialise optimizer state -- then the step is
    captured (try_capture: the decision is agreed across ranks) and every later call copies its
    batch into the static buffers and replays. A batch whose shape or layout differs (a ragged
    last batch; identical on every rank under DistributedSampler / even_batches) runs eagerly.
    ``capture=False`` (or no GPU) runs everything eagerly. The returned loss of a replay is the
    graph's static output tensor: read it before the next call."""

    def __init__(self, body, warmup: int = 2, capture: bool = True, log=print):
        self.body = body
        self.warmup = max(0, int(warmup))
        self.want = bool(capture) and torch.cuda.is_available()
        self.log = log
        self.sx = self.sy = None
        self.graph = None
        self.calls = 0
        self.replayed = 0
        self.eager = 0

    @property
    def captured(self) -> bool:
        return self.graph is not None

    def _eager(self, x, y):
        self.eager += 1
        return self.body(x, y)

    def __call__(self, x, y):
        self.calls += 1
        if not self.want:
            return self._eager(x, y)
        if self.sx is None:
            self.sx, self.sy = _static_like(x), _static_like(y)
        if _layout(x) != _layout(self.sx) or _layout(y) != _layout(self.sy):
            return self._eager(x, y)
        _fill(self.sx, x)
        _fill(self.sy, y)
        if self.graph is None:
            if self.calls <= self.warmup:
                return self._eager(self.sx, self.sy)
            g = try_capture(lambda: self.body(self.sx, self.sy), warmup=0, log=self.log)
            if not isinstance(g, CapturedStep):
                self.want = False
                return self._eager(self.sx, self.sy)
            self.graph = g
        self.replayed += 1
        return self.graph.replay()
