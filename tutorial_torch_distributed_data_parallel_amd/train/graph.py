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

import torch


class CapturedStep:
    def __init__(self, step_fn, warmup: int = 3, pool=None):
        if not torch.cuda.is_available():
            raise RuntimeError("CapturedStep needs a GPU")
        self.step_fn = step_fn
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):  # allocator warm-up, lazy kernel attributes, momentum init
                step_fn()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, pool=pool):
            self.output = step_fn()
        torch.cuda.synchronize()

    def replay(self):
        from ..optim.fused import sync_all_hyper

        sync_all_hyper()  # LR schedules etc. reach the captured kernels through the hyper blocks
        self.graph.replay()
        from ..parallel import runtime as rt

        comm = rt.comm()
        if comm is not None and comm.world > 1:
            comm.watch_current("captured training step")  # RCCL watchdog covers the replay
        return self.output

    __call__ = replay


def try_capture(step_fn, warmup: int = 3, log=print):
    """Capture if possible; on any capture error fall back to eager (returns step_fn)."""
    try:
        return CapturedStep(step_fn, warmup=warmup)
    except Exception as e:  # pragma: no cover - depends on runtime support
        log(f"[tdp] hipGraph capture failed, running eagerly: {e!r}")
        torch.cuda.synchronize()
        return step_fn
