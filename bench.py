#!/usr/bin/env python3
"""Flagship benchmark: toy-MLP DDP training throughput (samples/s for the whole node).

Metric / config from BASELINE.json: "samples/sec (whole node) toy-MLP DDP at 1/2/4/8 MI355X".
Model: ToyMLP 9216 -> 4096 -> 4096 -> 10 (Linear+ReLU; = the reference AlexNet's classifier),
per-rank batch 128 (REF/multi-GPU-training-torch.py:88), synthetic on-device data, random init,
fp32 (the reference's dtype), CrossEntropyLoss, SGD(momentum=0.9) (the north star's fused SGD),
one full DDP step per iteration: sampler-ordered batch gather -> forward -> loss -> backward with
bucketed RCCL gradient reduction -> optimizer step. Weak scaling: per-GPU work is fixed.

  python bench.py                                   # 1 GPU
  python bench.py --gpus N                          # N ranks, spawned by bench.py itself
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
  python bench.py --impl torch                      # stock torch DDP + torch.optim (comparison)
  python bench.py --api accelerate                  # the same step through Accelerator.prepare()

Execution: at world size > 1 the whole step is captured into a hipGraph and replayed, so the
bucket collectives run on the communicator's side stream and overlap backward (inside a graph the
cross-stream dependency is free; eagerly it slows every launch, profiles/side_stream_eager.md).
Optimizer scalars live in device hyper blocks, so the captured step stays exact (LR changes,
Adam's step count). At world size 1 the toy-MLP step is captured as well (no collective, the
optimizer runs in the weight-gradient GEMM epilogues; replay removes the host-side launch work
the ~15-kernel eager step is bound by); the CNNs run eagerly. ``--graph`` / ``--eager`` force a
mode. A captured toy-MLP replay runs FOUR training steps (``--graph-steps 4``, each with its own
batch gather and update; an epoch boundary always falls between replays), which pays the
graph-launch gap once per four steps; the trajectory is bit-identical to one step per replay.

Diagnostics (after the timed region, in the JSON line's "diagnostics"): at world size > 1 the
collectives of one step alone (``comm_ms``), the same captured step with its collectives turned
into no-ops (``compute_ms``), the share of the collective time hidden behind compute
(``overlap_pct``) and a short RCCL bus-bandwidth sweep; at world size 1 the single-GPU rehearsal
of the multi-GPU schedule (``rehearsal_ms``: RCCL collectives kept, per-bucket fused update,
captured step).

Timing: a device warm-up (``--device-warmup-ms`` of training steps on a scratch replica of the
model for the toy MLP, dummy GEMMs for the CNNs; ``--warmup-mode``) that touches no state of the
measured model,
then W untimed warm-up steps, then exactly K steps bracketed by barrier + device sync on
both sides; the max over ranks is reported; rank 0 prints one JSON line. Native libraries (RCCL
prints a version banner when a communicator is created) write to file descriptor 1, so the
process points fd 1 at stderr and writes the JSON line to a private duplicate of the original
stdout: stdout carries exactly one line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time
from pathlib import Path

import torch

METRIC = "samples/sec (whole node) toy-MLP DDP at 1/2/4/8 MI355X; scaling efficiency"
ROOT = Path(__file__).resolve().parent
# Bucket plan (csrc/reducer.cpp compute_bucket_bounds): DDP's 25 MiB cap and 1 MiB first bucket;
# a parameter larger than the cap is one bucket, and the small leftovers in front of it ride along
# (toy MLP: {fc3, fc2} 64.2 MiB ready after fc2's weight gradient, overlapping fc1's backward;
# {fc1} 144 MiB at the end) -- torch DDP's own post-rebuild plan, without its 1-MiB collectives.
# Splitting fc1 (--split-mb) buys no overlap: its whole gradient comes from one GEMM.
DIAG_SWEEP_MB = (1, 8, 32, 128)


def _private_stdout():
    """Return a writer on the original stdout and point fd 1 at stderr (see module doc)."""
    sys.stdout.flush()
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    return out


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=128, help="per-rank batch")
    ap.add_argument("--impl", choices=["tdp", "torch"], default="tdp")
    ap.add_argument("--api", choices=["ddp", "accelerate"], default="ddp",
                    help="tdp: drive the step through DDP directly, or through the Accelerate-style "
                         "Accelerator.prepare() facade (BASELINE.json config 4)")
    ap.add_argument("--optim", choices=["sgd", "adam"], default="sgd")
    ap.add_argument("--bucket-mb", type=float, default=None)
    ap.add_argument("--split-mb", type=float, default=None,
                    help="cut parameters larger than this into buckets of this size")
    ap.add_argument("--device-warmup-ms", type=float, default=200.0,
                    help="GPU clock warm-up (dummy GEMMs, no model state) before the W warm-up "
                         "steps; 0 = off (see device_warmup)")
    ap.add_argument("--warmup-mode", choices=["auto", "scratch", "gemm"], default="auto",
                    help="device warm-up before the W warm-up steps: training steps of a scratch "
                         "replica of the model (tdp) or dummy GEMMs; auto = scratch for the toy "
                         "MLP, GEMMs for the CNNs")
    ap.add_argument("--no-diag", action="store_true",
                    help="skip the post-measurement diagnostics (comm / compute / rehearsal)")
    ap.add_argument("--syncbn", action="store_true", help="toy MLP + SyncBatchNorm config")
    ap.add_argument("--model", choices=["toy_mlp", "alexnet", "resnet50"], default="toy_mlp",
                    help="toy_mlp = the headline config; alexnet / resnet50 = the CNN configs")
    ap.add_argument("--mlp-dims", type=str, default=None,
                    help="toy MLP in,hidden1,hidden2 (tests only; the headline is 9216,4096,4096)")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--dataset", type=int, default=None,
                    help="synthetic samples per rank (default 8192 MLP, 512 CNN)")
    ap.add_argument("--cpu", action="store_true", help="CPU/gloo plumbing config")
    ap.add_argument("--compression", choices=["none", "bf16"], default="none")
    ap.add_argument("--graph", action="store_true",
                    help="tdp: capture the whole step into a hipGraph and replay it (the default; "
                         "at world size > 1 the bucket collectives then overlap backward on the "
                         "comm stream)")
    ap.add_argument("--graph-steps", type=int, default=4,
                    help="training steps per captured hipGraph replay (G steps per graph pay "
                         "the graph-launch gap once per G steps; a group that would cross an "
                         "epoch boundary runs step by step)")
    ap.add_argument("--eager", action="store_true",
                    help="tdp: run eagerly (collectives then run on the compute stream without "
                         "overlap)")
    ap.add_argument("--fused-opt", choices=["auto", "on", "off"], default="auto",
                    help="tdp: apply the optimizer inside the gradient reduction (DDP "
                         "register_fused_optimizer): with world_size > 1 per bucket and sharded "
                         "(reduce-scatter -> update 1/W -> all-gather: same wire bytes, 1/W of "
                         "the optimizer's HBM traffic); with world_size 1 in the weight-gradient "
                         "GEMM epilogues (no gradient write/re-read). auto = on")
    ap.add_argument("--no-fused-opt", action="store_true", help="alias of --fused-opt off")
    ap.add_argument("--parallel", choices=["ddp", "auto", "tensor"], default="ddp",
                    help="N > 1 toy MLP: 'ddp' (default, the headline) = the DDP reducer's "
                         "ladder, recorded as dp{N}; 'tensor' = the tensor-sharded step "
                         "(parallel/tensor_parallel.py: activations cross xGMI, not weights; not "
                         "DDP), recorded as tp{N}; 'auto' = the DDP headline plus the "
                         "tensor-sharded variants' timings as side numbers in config.selection")
    ap.add_argument("--tp-replicated-data", action="store_true",
                    help="--parallel tensor: every rank holds the whole dataset and gathers the "
                         "node's batch locally instead of all-gathering the ranks' inputs")
    ap.add_argument("--select-steps", type=int, default=20,
                    help="timed steps per candidate of --parallel tensor / auto")
    ap.add_argument("--head-loss", choices=["fused", "separate"], default="separate",
                    help="toy MLP: the head Linear + cross-entropy as the reference's two calls "
                         "(criterion(model(x), y), default) or as one fused op (model(x, "
                         "target=y): ops.linear_cross_entropy, one launch for the head GEMM, the "
                         "loss and the head's input gradient); bit-identical results, measured at "
                         "parity (profiles/r10/head_ce_r10.md)")
    ap.add_argument("--comm-cus", type=int, default=None,
                    help="CUs left to RCCL: grid-sized kernels (persistent GEMMs, split-K "
                         "planners) plan for (CUs - N) (TDP_COMM_CUS; default 0)")
    return ap.parse_args()


def baseline_for(n_gpus: int, impl: str, syncbn: bool, model: str = "toy_mlp"):
    """(samples/s, source) of stock torch DDP + torch.optim on MI355X for the same config
    (bench_baseline.json), or (None, None). Without a measured N-GPU stock row (the development
    box has one GPU) the baseline at N > 1 is the measured 1-GPU stock number times N: stock DDP
    with PERFECT scaling, an upper bound of the real stock figure, so vs_baseline understates
    this framework's advantage rather than inflating it."""
    f = ROOT / "bench_baseline.json"
    if impl != "tdp" or not f.exists() or not torch.cuda.is_available():
        return None, None
    try:
        tab = json.loads(f.read_text())
        name = {"toy_mlp": "mlp"}.get(model, model)
        stem = f"{name}{'_syncbn' if syncbn else ''}_dp"
        v = tab.get(f"{stem}{n_gpus}")
        if v:
            return float(v), f"bench_baseline.json {stem}{n_gpus} (measured)"
        v1 = tab.get(f"{stem}1")
        if v1 and n_gpus > 1:
            return float(v1) * n_gpus, (f"bench_baseline.json {stem}1 x {n_gpus} (stock 1-GPU "
                                        "number with perfect scaling: an upper bound)")
        return None, None
    except Exception:
        return None, None


MODEL_DESC = {
    "toy_mlp": "toy-MLP {dims} (Linear+ReLU{bn})",
    "alexnet": "AlexNet (torchvision topology, 10 classes, 3x{s}x{s}{bn})",
    "resnet50": "ResNet-50 (torchvision v1.5 topology, 10 classes, 3x{s}x{s}{bn})",
}


def _gemm_products(impl: str, use_gpu: bool):
    """How the fp32 GEMMs form their products (tdp fast GEMM: csrc/gemm_f32_fast.hip)."""
    if impl != "tdp" or not use_gpu:
        return None
    from tutorial_torch_distributed_data_parallel_amd._native import native

    if native().gemm_f32_emu():
        return ("fp32 operands split exactly into 3 bf16 terms (RNE), 6 bf16 MFMA products with "
                "fp32 accumulation: error within the native f32 bound (tests/test_gemm_emu_gpu.py)")
    return "native v_mfma_f32_32x32x2_f32"


def _reserved_cus(impl: str, use_gpu: bool):
    if impl != "tdp" or not use_gpu:
        return None
    from tutorial_torch_distributed_data_parallel_amd._native import native

    return int(native().reserved_cus())


def scratch_warmup(a, dims, in_shape, dev):
    """Device warm-up on a SCRATCH replica of the benchmarked model (same architecture, its own
    random weights, optimizer and random batch; no DDP, no collectives, nothing shared with the
    measured model): ``--device-warmup-ms`` of real training steps before the W warm-up steps.
    Motivation (profiles/micro/bench_warmup_r4o.txt): after 200 ms of dummy GEMMs a 20-step
    window ran at 0.401 ms/step against 0.375 for steps 20-119 (1000 ms of GEMMs: 0.398); the
    window length, not the dataset, matters (bench_warmup_r4q.txt). With the scratch replica the
    20-step toy-MLP window ran at 0.385-0.391 vs 0.396-0.408 (r4p round 1, r4q; r4p round 2 was a
    noisy box); the CNNs do not move, so ``auto`` uses it for the toy MLP only."""
    import tutorial_torch_distributed_data_parallel_amd as tdp
    from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP
    from tutorial_torch_distributed_data_parallel_amd.models.registry import build_model

    if a.device_warmup_ms <= 0:
        return
    g = torch.Generator(device=dev).manual_seed(7)
    if a.model == "toy_mlp":
        m = ToyMLP(in_features=dims[0], hidden=dims[1:], batchnorm=a.syncbn, device=dev)
    else:
        m = build_model(a.model, device=dev)
    opt = (tdp.optim.SGD(m.parameters(), lr=0.01, momentum=0.9) if a.optim == "sgd"
           else tdp.optim.Adam(m.parameters(), lr=1e-3))
    x = torch.randn((a.batch,) + tuple(in_shape), device=dev, generator=g)
    if x.dim() == 4:
        x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (a.batch,), device=dev, generator=g)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1000.0 < a.device_warmup_ms:
        for _ in range(4):
            opt.zero_grad(set_to_none=True)
            tdp.ops.backward(tdp.ops.cross_entropy(m(x), y))
            opt.step()
        torch.cuda.synchronize()
    del m, opt, x, y


def device_warmup(dev, ms: float, native_gemm: bool):
    """Bring the GPU to its steady-state clock before the W warm-up steps: ``ms`` of dummy
    2048^3 GEMMs (no model state is touched). Measured on MI355X (scripts/step_timeline.py,
    profiles/bench_clock_ramp_r3.md): from a cold start the toy-MLP step needs ~40 steps (~20 ms
    of load) to settle -- 0.49 ms for steps 10-19, 0.476 for 20-29, 0.455 from step 40 on -- so a
    5-step warm-up timed the power-management ramp instead of the training step. Both --impl
    variants get the same warm-up."""
    if ms <= 0:
        return
    a = torch.randn(2048, 2048, device=dev)
    b = torch.randn(2048, 2048, device=dev)
    c = torch.empty(2048, 2048, device=dev)
    if native_gemm:
        from tutorial_torch_distributed_data_parallel_amd._native import native

        C = native()
        run = lambda: C.gemm_f32(a, b, c, True, True)  # noqa: E731
    else:
        run = lambda: torch.mm(a, b.t(), out=c)  # noqa: E731
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1000.0 < ms:
        for _ in range(16):
            run()
        torch.cuda.synchronize()
    del a, b, c


def _time_steps(step, n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1000.0 / n


def predicted_comm(a, ddp, world, sweep) -> dict:
    """The step model (parallel/commmodel.py, docs/COMM_MODEL.md) fed with this job's measured
    bus bandwidths (largest swept size per collective) and its sync plan: the exposed
    communication it predicts, reported next to the measured overlap."""
    from tutorial_torch_distributed_data_parallel_amd.parallel import commmodel as cm

    big = {}
    for r in sweep:
        if r["bytes"] >= big.get(r["op"], (0, 0))[0]:
            big[r["op"]] = (r["bytes"], r["busbw_GBps"])
    hw = cm.Hardware(busbw_GBps={op: bw for op, (_, bw) in big.items()})
    dims = tuple(int(v) for v in a.mlp_dims.split(",")) if a.mlp_dims else (9216, 4096, 4096)
    layers = cm.toy_mlp_layers(a.batch, dims)
    plan = ddp.sync_plan()
    modes = {}
    for name in ("fc1", "fc2"):
        m = plan.get(f"{name}.weight", "allreduce")
        modes[name] = m if m in cm.MODES else "allreduce"
    r = cm.simulate(layers, modes, world, a.batch, hw)
    return {"predicted_comm_exposed_ms": round(r["exposed_us"] / 1000.0, 4),
            "predicted_step_ms": round(r["step_us"] / 1000.0, 4),
            "predicted_modes": modes}


def diagnostics(a, ddp, step, step_ms, world, graph, barrier, build_rehearsal):
    """Post-measurement evidence for the scaling curve (module doc). Every rank runs the same
    collectives in the same order; rank 0 reports."""
    from tutorial_torch_distributed_data_parallel_amd.parallel import commbench
    from tutorial_torch_distributed_data_parallel_amd.parallel import runtime as rt
    from tutorial_torch_distributed_data_parallel_amd.train.graph import try_capture

    n = max(10, min(a.steps, 50))
    out = {"mode": "graph" if graph else "eager"}
    if world > 1 or os.environ.get("TDP_DIAG_MULTI") == "1":  # (the latter: test at world 1)
        comm_ms = commbench.ddp_comm_ms(ddp, iters=10)
        # the same step with its collectives turned into no-ops (re-captured when graphed)
        ddp._ops.skip_collectives = True
        try:
            st = step
            if graph:
                st = try_capture(getattr(step, "raw", step), warmup=2, log=lambda m: None)
            barrier()
            compute_ms = _time_steps(st, n)
        finally:
            ddp._ops.skip_collectives = False
        t = torch.tensor([comm_ms, compute_ms], dtype=torch.float64, device=rt.device())
        rt.all_reduce(t, "max")
        comm_ms, compute_ms = (float(v) for v in t.tolist())
        # share of the collective time that ran concurrently with compute
        hidden = max(0.0, comm_ms + compute_ms - step_ms)
        out.update(comm_ms=round(comm_ms, 4), compute_ms=round(compute_ms, 4),
                   overlap_pct=round(100.0 * min(hidden, comm_ms) / comm_ms, 1)
                   if comm_ms > 0 else None)
        sweep = commbench.collective_busbw([m * 2 ** 20 for m in DIAG_SWEEP_MB], iters=5,
                                           warmup=2)
        out["busbw_GBps"] = {f"{r['op']}@{r['bytes'] >> 20}MiB": r["busbw_GBps"] for r in sweep}
        if a.model == "toy_mlp":
            out.update(predicted_comm(a, ddp, world, sweep))
    elif build_rehearsal is not None:
        from tutorial_torch_distributed_data_parallel_amd.train.graph import CapturedStep

        d2, st1 = build_rehearsal()
        # the timed step's replay form: G training steps per graph launch when the measured
        # step ran that way (a W > 1 bench captures the same G-step graph), so the ratio to dp1
        # compares schedules, not graph-launch counts
        G = max(1, int(getattr(step, "graph_steps", 1) or 1))

        def st():
            for _ in range(G):
                st1()
        reps = max(1, n // G)
        g = CapturedStep(st, warmup=3)
        out["rehearsal_ms"] = round(_time_steps(g.replay, reps) / G, 4)
        out["rehearsal_buckets"] = len(d2._bounds) - 1
        out["rehearsal_graph_steps"] = G
        del g
        # the same schedule with its one-rank collectives turned into no-ops: at world size 1 an
        # all-gather / reduce-scatter is a local copy on the comm queue (factors, buckets) that
        # competes for HBM with the compute stream -- traffic a W-rank job moves over xGMI
        # instead. What remains over dp1 is the schedule itself (side-stream forks and joins,
        # per-bucket / factored updates instead of the GEMM epilogue).
        d2._ops.skip_collectives = True
        try:
            g = CapturedStep(st, warmup=2)
            out["rehearsal_schedule_ms"] = round(_time_steps(g.replay, reps) / G, 4)
            del g
        finally:
            d2._ops.skip_collectives = False
        out["rehearsal_over_dp1"] = round(out["rehearsal_ms"] / step_ms, 4)
        out["rehearsal_schedule_over_dp1"] = round(out["rehearsal_schedule_ms"] / step_ms, 4)
        del d2
        if a.model == "toy_mlp" and not a.syncbn and a.api == "ddp":
            # the tensor-sharded step's per-rank compute at W = 2 / 8 on this GPU (shard
            # shapes, collectives as local copies) and the step it predicts with the assumed
            # xGMI figures (docs/COMM_MODEL.md "Tensor-sharded")
            from tutorial_torch_distributed_data_parallel_amd.parallel import commmodel as cm
            from tutorial_torch_distributed_data_parallel_amd.parallel.tensor_parallel import \
                rank_compute_ms

            dims = tuple(int(v) for v in a.mlp_dims.split(",")) if a.mlp_dims else \
                (9216, 4096, 4096)
            rk, pred = {}, {}
            for W in (2, 8):
                # (>= 200 replays: a 20-step window read 4-7 % high against the proxy's)
                ms = rank_compute_ms(W, dims=dims, B=a.batch, steps=max(n, 200), optim=a.optim)
                rk[str(W)] = round(ms, 4)
                pred[str(W)] = round(cm.simulate_tensor(W, B=a.batch, dims=dims,
                                                        rank_us=ms * 1000.0, chunks=2)
                                     ["step_us"] / 1000.0, 4)
            out["tensor_rank_compute_ms"] = rk
            # the rehearsal of the execution --parallel auto can pick at N > 1 (per-rank compute
            # of the tensor-sharded step over dp1; the DDP schedule's is rehearsal_over_dp1)
            out["tensor_rank_over_dp1"] = {k: round(v / step_ms, 4) for k, v in rk.items()}
            out["tensor_predicted_step_ms"] = pred
            out["tensor_predicted_eff"] = {k: round(step_ms / v, 3) for k, v in pred.items()}
    return out


def tensor_diagnostics(a, job, step_ms, world, barrier):
    """N > 1, tensor-sharded step measured: the same step with every collective replaced by its
    local copy (re-captured; rank 0's shard shapes on every rank) = this rank's compute; the
    exposed communication is the measured step minus it. Plus the RCCL bus-bandwidth sweep and
    the model's prediction from it (docs/COMM_MODEL.md "Tensor-sharded")."""
    from tutorial_torch_distributed_data_parallel_amd.parallel import commbench
    from tutorial_torch_distributed_data_parallel_amd.parallel import commmodel as cm
    from tutorial_torch_distributed_data_parallel_amd.parallel import runtime as rt
    from tutorial_torch_distributed_data_parallel_amd.parallel import tensor_parallel as TPm
    from tutorial_torch_distributed_data_parallel_amd.train.graph import try_capture

    n = max(10, min(a.steps, 50))
    out = {"mode": "graph" if job.graph else "eager", "execution": job.rung}
    TPm.set_fake_world(world)
    try:
        st = getattr(job.step, "raw", job.step)
        if job.graph:
            st = try_capture(st, warmup=2, log=lambda m: None)
        barrier()
        compute_ms = _time_steps(st, n)
    finally:
        TPm.set_fake_world(0)
    t = torch.tensor([compute_ms], dtype=torch.float64, device=rt.device())
    rt.all_reduce(t, "max")
    compute_ms = float(t.item())
    out.update(compute_ms=round(compute_ms, 4), exposed_comm_ms=round(step_ms - compute_ms, 4))
    sweep = commbench.collective_busbw([m * 2 ** 20 for m in DIAG_SWEEP_MB], iters=5, warmup=2)
    out["busbw_GBps"] = {f"{r['op']}@{r['bytes'] >> 20}MiB": r["busbw_GBps"] for r in sweep}
    big = {}
    for r in sweep:
        if r["bytes"] >= big.get(r["op"], (0, 0))[0]:
            big[r["op"]] = (r["bytes"], r["busbw_GBps"])
    dims = tuple(int(v) for v in a.mlp_dims.split(",")) if a.mlp_dims else (9216, 4096, 4096)
    hw = cm.Hardware(busbw_GBps={op: bw for op, (_, bw) in big.items()})
    pred = cm.simulate_tensor(world, B=a.batch, dims=dims, hw=hw, rank_us=compute_ms * 1e3,
                              chunks=int(job.tp.overlap_chunks),
                              global_batch=bool(a.tp_replicated_data))
    out.update(predicted_step_ms=round(pred["step_us"] / 1e3, 4),
               predicted_exposed_ms=round(pred["exposed_us"] / 1e3, 4))
    return out


def _launcher_env() -> bool:
    """True when a launcher (torchrun, parallel/launcher.py, this script's own parent) already
    made this process one rank of a job."""
    return "RANK" in os.environ or "LOCAL_RANK" in os.environ


def _multi_rank_vehicle() -> str | None:
    """Several ranks may share one GPU only through an explicit vehicle (parallel/relay.py,
    parallel/peer.py); RCCL refuses duplicate devices."""
    if os.environ.get("TDP_GPU_PEER", "0") == "1":
        return "peer"
    if os.environ.get("TDP_GPU_RELAY", "0") == "1":
        return "relay"
    return None


def launched_by() -> str:
    if os.environ.get("TDP_BENCH_LAUNCHED_BY"):
        return os.environ["TDP_BENCH_LAUNCHED_BY"]
    if "TORCHELASTIC_RUN_ID" in os.environ:
        return "torch.distributed.run"
    return "external launcher" if _launcher_env() else "direct (one process)"


def self_launch(a) -> int:
    """``python bench.py --gpus N`` (N > 1) with no launcher environment: this process becomes
    the launcher (the reference spawns its ranks from the configured world size itself,
    REF/multi-GPU-training-torch.py:269-279,306). It never touches the GPU -- counting devices
    does not initialise HIP on this image -- and never re-executes itself: the N ranks are child
    processes (parallel/launcher.run_script, fail-fast), rank 0's stdout comes back through a
    file, and its single JSON line is checked (n_gpus / parallelism = N) and relayed. Exit code:
    the first failing rank's, 3 for a malformed record, 2 when fewer than N GPUs are visible and
    no one-GPU vehicle was asked for."""
    import tempfile

    from tutorial_torch_distributed_data_parallel_amd.parallel.launcher import run_script

    n = a.gpus
    if not a.cpu:
        have = torch.cuda.device_count()
        if have < n and _multi_rank_vehicle() is None:
            print(f"bench.py: --gpus {n} but only {have} GPU(s) are visible; refusing to report "
                  f"a {n}-rank number (TDP_GPU_PEER=1 / TDP_GPU_RELAY=1 run several ranks on one "
                  f"GPU for testing)", file=sys.stderr, flush=True)
            return 2
    how = f"bench.py (self-launched {n} ranks, parallel/launcher.run_script)"
    with tempfile.TemporaryFile(mode="w+") as f0:
        rc = run_script(n, [str(Path(__file__).resolve()), *sys.argv[1:]],
                        env_extra={"TDP_BENCH_LAUNCHED_BY": how}, rank0_stdout=f0)
        f0.seek(0)
        lines = [ln for ln in f0.read().splitlines() if ln.strip()]
    if rc != 0:
        print(f"bench.py: a rank failed with exit code {rc}", file=sys.stderr, flush=True)
        for ln in lines:
            print(ln, file=sys.stderr)
        return rc if rc > 0 else 1
    try:
        rec = json.loads(lines[-1])
        want_n = n if not a.cpu else 0
        ok = rec["n_gpus"] == want_n and rec["config"]["parallelism"] in (f"dp{n}", f"tp{n}")
    except Exception:  # noqa: BLE001 - anything unparsable is a malformed record
        ok, rec = False, None
    if not ok:
        print(f"bench.py: rank 0 printed no valid {n}-rank record: {lines[-3:]}",
              file=sys.stderr, flush=True)
        return 3
    print(json.dumps(rec), flush=True)
    return 0


class BenchFault:
    """TDP_BENCH_FAULT="name[,name...]" (tests of the fallback ladder): make that rung fail on
    EVERY rank, at the first attempt only ("name@*": at every attempt). Names: ``tune`` (the
    factored-mode tuning raises), ``factored`` (setup with factored weights raises), ``fused``
    (setup with a fused optimizer raises), ``warmup`` (the first warm-up step raises). A capture
    failure on one rank is TDP_FAULT_CAPTURE=<rank> (train/graph.py)."""

    def __init__(self):
        spec = [t.strip() for t in os.environ.get("TDP_BENCH_FAULT", "").split(",") if t.strip()]
        self.once = {t for t in spec if not t.endswith("@*")}
        self.always = {t[:-2] for t in spec if t.endswith("@*")}

    def check(self, name: str, attempt: int) -> None:
        if name in self.always or (name in self.once and attempt == 0):
            raise RuntimeError(f"injected bench fault '{name}' (TDP_BENCH_FAULT)")


# The fallback ladder at world size > 1: the first real N-GPU run must yield
# a number, not a crash. Every rung is tried on every rank; a failure anywhere (setup, tuning,
# warm-up steps) is agreed over all ranks (a host-side MIN all-reduce) and every rank moves to the
# next rung together. Rung 0 is the full schedule; the last is the reference's own step (plain
# bucketed all-reduce, optimizer.step(), eager). Inside a rung: a failed factored-mode tuning keeps
# the model's choice, a failed capture runs that rung eagerly (both agreed, recorded).
LADDER = (
    {"name": "full", "factor": None, "fused": True, "graph": True},
    {"name": "sharded-buckets", "factor": False, "fused": True, "graph": True},
    {"name": "allreduce+optimizer.step", "factor": False, "fused": False, "graph": True},
    {"name": "eager-allreduce", "factor": False, "fused": False, "graph": False},
)


# The tensor-sharded step (parallel/tensor_parallel.py), opt-in: with --parallel tensor the faster
# of these is measured and recorded as tp{N} (it is not DDP: SURVEY.md section 2.4 lists DDP as
# the reference's only strategy); with --parallel auto they are timed as side numbers only.
TENSOR_RUNGS = (
    {"name": "tensor-sharded", "factor": None, "fused": True, "graph": True, "tensor": 1},
    # fc2's reduce-scatter / all-gather in column chunks behind the chunk GEMMs
    {"name": "tensor-overlap", "factor": None, "fused": True, "graph": True, "tensor": 2},
)


def _report_local(name: str, e: BaseException) -> None:
    """The failing rank's own traceback, printed BEFORE the agreement collective: when only some
    ranks fail, the others may be inside a collective of the rung and the agreement never lands
    (the watchdog then ends the job), so this line is the only record of the cause."""
    import traceback

    r = os.environ.get("RANK", "0")
    print(f"[bench] rank {r}: {name} raised:\n{traceback.format_exc()}", file=sys.stderr,
          flush=True)


def _agree(ok: bool) -> bool:
    from tutorial_torch_distributed_data_parallel_amd.train.graph import agree

    return agree(ok)


def build_tdp(a, ctx, cfg, attempt, fallbacks, fault):
    """One rung's job: model, DDP (or the Accelerate facade), optimizer, data, step closures,
    tuning and capture. Returns a namespace the caller times; raises on failure."""
    import types

    import tutorial_torch_distributed_data_parallel_amd as tdp
    from tutorial_torch_distributed_data_parallel_amd.data import (DeviceLoader,
                                                                    DistributedSampler,
                                                                    SyntheticDataset)
    from tutorial_torch_distributed_data_parallel_amd.data.synthetic import (
        EpochCursor, gather_batch, gather_batch_cursor)
    from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP
    from tutorial_torch_distributed_data_parallel_amd.models.registry import build_model

    dims, in_shape, use_gpu = ctx.dims, ctx.in_shape, ctx.use_gpu
    rank, world, dev = ctx.rank, ctx.world, ctx.dev
    graph = ctx.graph and cfg["graph"]
    torch.manual_seed(1234 + rank)
    if a.model == "toy_mlp":
        model = ToyMLP(in_features=dims[0], hidden=dims[1:], batchnorm=a.syncbn, device=dev)
    else:
        model = build_model(a.model, device=dev)
    if a.syncbn:
        model = tdp.nn.convert_sync_batchnorm(model)
    bucket_mb = a.bucket_mb
    fused = False

    def make_opt(params):
        if a.optim == "sgd":
            return tdp.optim.SGD(params, lr=0.01, momentum=0.9)
        return tdp.optim.Adam(params, lr=1e-3)

    # auto = on: world > 1 shards the update inside the reduction; world 1 applies it in
    # the weight-gradient GEMM epilogues (the local gradient is already the average)
    want_fused = a.fused_opt in ("on", "auto") and not a.no_fused_opt and cfg["fused"]
    acc = torch.zeros(3, device=dev)
    factor_kw = {} if cfg["factor"] is None else {"factor_sync": cfg["factor"]}

    def loss_fn(out_, y):
        return tdp.ops.cross_entropy(out_, y, acc=acc)

    # the toy MLP's head and loss as ONE op (models/mlp.py forward(x, target)): the same
    # criterion(model(inputs), labels) (REF/multi-GPU-training-torch.py:121-122), bit for bit
    fused_head = a.model == "toy_mlp" and a.head_loss == "fused"

    def model_loss(mod, x, y):
        if fused_head:
            return mod(x, target=y, acc=acc)
        return loss_fn(mod(x), y)

    tp = None
    bsz = a.batch  # rows one step gathers (the tensor-sharded step: the node's batch)
    if cfg.get("tensor"):
        from tutorial_torch_distributed_data_parallel_amd.parallel.tensor_parallel import \
            TensorParallelMLP

        if a.model != "toy_mlp" or a.api != "ddp":
            raise RuntimeError("tensor-sharded step: the toy MLP through the native DDP API only")
        # default: each rank gathers its own batch (its DistributedSampler share) and the
        # wrapper all-gathers the node's inputs over xGMI (33 MB per step at W = 8), as a real
        # per-rank input pipeline would. --tp-replicated-data: every rank holds the whole
        # dataset and every rank's sampler and gathers the node's batch from its own HBM (a
        # data-layout assumption the DDP path does not make; recorded in config.tp_data)
        shared = bool(a.tp_replicated_data)
        tp = TensorParallelMLP(model, global_batch=shared, overlap_chunks=int(cfg["tensor"]))
        ddp = None
        opt = make_opt(tp.parameters())
        if use_gpu and want_fused:
            # the shards' SGD inside their weight-gradient GEMMs (complete gradients per rank)
            fused = tp.register_fused_optimizer(opt)
        if shared:
            data = SyntheticDataset(a.dataset * world, in_shape, 10, seed=0, device=dev)
            samplers = [DistributedSampler(data, num_replicas=world, rank=r, shuffle=True)
                        for r in range(world)]
            loaders = [DeviceLoader(data, a.batch, sampler=s_, drop_last=True)
                       for s_ in samplers]

            class _NodeOrder:
                """The node's batch order: step s = rank 0's batch s, rank 1's batch s, ..."""

                def set_epoch(self, e):
                    for s_ in samplers:
                        s_.set_epoch(e)

                def epoch_indices(self):
                    idx = torch.stack([ld.epoch_indices() for ld in loaders])
                    nb = idx.shape[1] // a.batch
                    return idx[:, :nb * a.batch].reshape(world, nb, a.batch).transpose(0, 1) \
                        .reshape(-1).contiguous()
            sampler = loader = _NodeOrder()
            bsz = a.batch * world
            own = slice(rank * a.batch, (rank + 1) * a.batch)
        else:
            data = SyntheticDataset(a.dataset, in_shape, 10, seed=rank, device=dev)
            sampler = DistributedSampler(data, num_replicas=world, rank=rank, shuffle=True)
            loader = DeviceLoader(data, a.batch, sampler=sampler, drop_last=True)
            own = slice(None)

        def body(x, y):  # REF/multi-GPU-training-torch.py:118-126, sharded execution
            opt.zero_grad(set_to_none=True)
            loss = loss_fn(tp(x), y[own])
            tdp.ops.backward(loss)
            tp.sync_grads()  # the replicated head / bias: averaged all-reduce
            opt.step()
            return loss
    elif a.api == "accelerate":
        # BASELINE.json config 4: the step through the Accelerate-style facade. One dataset
        # shared by all ranks, dealt out by whole batches (Accelerate's BatchSamplerShard).
        from tutorial_torch_distributed_data_parallel_amd.accelerate import Accelerator

        accel = Accelerator(ddp_kwargs=dict(bucket_cap_mb=bucket_mb, **factor_kw))
        opt = make_opt(model.parameters())
        data = SyntheticDataset(a.dataset * world, in_shape, 10, seed=0, device=dev)
        loader = DeviceLoader(data, a.batch, drop_last=True)
        model, opt, loader = accel.prepare(model, opt, loader)
        # the prepared model's DDP: the wrapper at N > 1, the hidden world-1 DDP of the
        # unwrapped one-process model (Accelerator.ddp_of)
        ddp = accel.ddp_of(model)
        if use_gpu and want_fused and ddp is not None:
            fused = accel.fuse_optimizer(model, opt)
        sampler = loader  # set_epoch lives on the prepared loader

        def body(x, y):  # REF/multi-GPU-training-accelerate.py:45-55
            opt.zero_grad(set_to_none=True)
            loss = model_loss(model, x, y)
            accel.backward(loss)
            opt.step()
            return loss
    else:
        ddp = tdp.DDP(model, device_ids=[dev.index] if use_gpu else None,
                      bucket_cap_mb=bucket_mb, split_bucket_mb=a.split_mb,
                      grad_compression=None if a.compression == "none" else a.compression,
                      **factor_kw)
        opt = make_opt(ddp.parameters())
        if use_gpu and want_fused:
            fused = ddp.register_fused_optimizer(opt)
        data = SyntheticDataset(a.dataset, in_shape, 10, seed=rank, device=dev)
        sampler = DistributedSampler(data, num_replicas=world, rank=rank, shuffle=True)
        loader = DeviceLoader(data, a.batch, sampler=sampler, drop_last=True)

        def body(x, y):  # REF/multi-GPU-training-torch.py:118-126
            opt.zero_grad(set_to_none=True)
            loss = model_loss(ddp, x, y)
            tdp.ops.backward(loss)  # loss.backward() seeded by a cached 1: no fill kernel
            opt.step()
            return loss
    if fused:
        fault.check("fused", attempt)
    if ddp is not None and ddp._factor:
        fault.check("factored", attempt)

    def build_rehearsal():
        """World size 1: the multi-GPU schedule on one GPU (RCCL collectives kept at world
        size 1, per-bucket fused update instead of the GEMM epilogue, captured step)."""
        torch.manual_seed(99)
        m2 = (ToyMLP(in_features=dims[0], hidden=dims[1:], batchnorm=a.syncbn, device=dev)
              if a.model == "toy_mlp" else build_model(a.model, device=dev))
        if a.syncbn:
            m2 = tdp.nn.convert_sync_batchnorm(m2)
        d2 = tdp.DDP(m2, device_ids=[dev.index], bucket_cap_mb=bucket_mb,
                     split_bucket_mb=a.split_mb, force_collective=True)
        o2 = make_opt(d2.parameters())
        if want_fused:
            d2.register_fused_optimizer(o2)

        def st():
            x, y = gather_batch(data.x, data.y, idx_static)
            o2.zero_grad(set_to_none=True)
            tdp.ops.backward(model_loss(d2, x, y))
            o2.step()
        return d2, st

    # batches are gathered on the device by the sampler's indices (one H2D copy per epoch);
    # a captured graph reads them from a static index tensor, eager steps from a slice
    idx_static = torch.empty(bsz, dtype=torch.long, device=dev)
    cur = {"epoch": 0, "pos": 0, "idx": loader.epoch_indices(), "b": None}
    idx_static.copy_(cur["idx"][:bsz])
    # captured toy-MLP step: the gather reads the epoch order through a device-side cursor
    # it advances itself (no per-step index copy node in the graph)
    ecur = None
    if graph and use_gpu and EpochCursor.fits(data.x, data.y, bsz):
        ecur = EpochCursor(len(cur["idx"]), bsz, dev)
        ecur.set_order(cur["idx"])

    def advance():
        if cur["pos"] + bsz > len(cur["idx"]):
            cur["epoch"] += 1
            sampler.set_epoch(cur["epoch"])
            cur["idx"], cur["pos"] = loader.epoch_indices(), 0
            if ecur is not None:
                ecur.set_order(cur["idx"])
        b = cur["idx"][cur["pos"]: cur["pos"] + bsz]
        if graph and ecur is None:
            idx_static.copy_(b)
            b = idx_static
        cur["b"] = b
        cur["pos"] += bsz

    def tdp_step():
        if ecur is not None:
            x, y = gather_batch_cursor(data.x, data.y, ecur)
            return body(x, y)
        b = idx_static if graph else cur["b"]
        x, y = gather_batch(data.x, data.y, b)
        return body(x, y)

    advance()
    run = tdp_step
    run_pair = [None]  # the G-step graph, when captured
    if ddp is not None and world > 1 and use_gpu:
        # measured replicated-vs-sharded choice per factored Linear weight (untimed training
        # steps, agreed over ranks) before the step is captured -- timed the way the step
        # will run: captured and replayed when the bench captures it
        def eager_step():
            advance()
            x, y = gather_batch(data.x, data.y, cur["b"])
            return body(x, y)
        # also: 0 or 8 CUs left free for RCCL's kernels while the persistent epilogue GEMMs
        # run (profiles/micro/comm_cus_ab.txt: 8 cost 3 % at dp1, whether they pay at N > 1
        # only the real node can tell), unless --comm-cus fixed it
        cus = (0, 8) if a.comm_cus is None else None
        from tutorial_torch_distributed_data_parallel_amd._native import native

        cus0 = int(native().reserved_cus())
        ok, err = True, None
        try:
            fault.check("tune", attempt)
            if graph:
                ddp.tune_factor_replicate(tdp_step, iters=20, capture=True, comm_cus=cus,
                                          repeats=2)
            else:
                ddp.tune_factor_replicate(eager_step, iters=3, comm_cus=cus)
        except Exception as e:  # noqa: BLE001 - the ladder's first rung: keep the model's choice
            ok, err = False, e
            _report_local(f"{cfg['name']}: factored-mode tuning", e)
        if not _agree(ok):
            # every rank drops the tuning result alike: the auto rule decides each weight
            native().set_reserved_cus(cus0)
            ddp.factor_replicate = None
            ddp.factor_tuning = None
            if hasattr(ddp, "consolidate_optimizer_state"):
                ddp.consolidate_optimizer_state()
            fallbacks.append(f"{cfg['name']}: factored-mode tuning failed "
                             f"({repr(err)[:160] if err else 'on another rank'}); kept the "
                             "model's choice")
    if graph:
        from tutorial_torch_distributed_data_parallel_amd.train.graph import (CapturedStep,
                                                                              try_capture)

        run = try_capture(tdp_step, warmup=3,
                          log=lambda m: print(m, file=sys.stderr, flush=True))
        if not isinstance(run, CapturedStep):
            fallbacks.append(f"{cfg['name']}: hipGraph capture failed (agreed over ranks); "
                             "the step runs eagerly")
        G = max(1, int(a.graph_steps))
        if ecur is not None and G > 1 and isinstance(run, CapturedStep):
            # G training steps per replay (the device cursor advances per gather): 1/G of the
            # graph launches; every step still runs all of its work
            def g_steps():
                out = None
                for _ in range(G):
                    out = tdp_step()
                return out
            # no eager warm-up: the one-step graph's warm-up already did it, and training
            # steps outside the count would make the run differ from --graph-steps 1
            run2 = try_capture(g_steps, warmup=0,
                               log=lambda m: print(m, file=sys.stderr, flush=True))
            if run2 is not g_steps:
                run_pair[0] = run2
        if ecur is not None:
            # the warm-up / capture runs advanced the device cursor: restart the epoch's
            # order so host and device positions agree from the first timed step on
            ecur.set_order(cur["idx"])
            cur["pos"] = 0

    def step():
        advance()
        return run()

    def steps(n):
        """n training steps; groups of G through the G-step graph while they fall in the
        current epoch (the host advances its position for each)."""
        k, out = 0, None
        while k < n:
            G = a.graph_steps
            if run_pair[0] is not None and n - k >= G and \
                    cur["pos"] + G * bsz <= len(cur["idx"]):
                for _ in range(G):
                    advance()
                out = run_pair[0]()
                k += G
            else:
                out = step()
                k += 1
        return out
    step.raw = tdp_step  # the uncaptured body (diagnostics re-capture it)
    step.many = steps
    step.graph_steps = a.graph_steps if run_pair[0] is not None else (1 if graph else 0)
    return types.SimpleNamespace(ddp=ddp, tp=tp, opt=opt, fused=fused, step=step, run=run,
                                 graph=graph, rung=cfg["name"],
                                 build_rehearsal=None if (a.api == "accelerate" or tp is not None)
                                 else build_rehearsal)


def main():
    a = parse()
    if a.gpus > 1 and not _launcher_env():
        sys.exit(self_launch(a))
    out = _private_stdout()
    if a.dataset is None:
        a.dataset = 8192 if a.model == "toy_mlp" else 512
    dims = tuple(int(v) for v in a.mlp_dims.split(",")) if a.mlp_dims else (9216, 4096, 4096)
    metric = METRIC if a.model == "toy_mlp" else \
        f"samples/sec (whole node) {a.model} DDP at 1/2/4/8 MI355X"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus and "RANK" in os.environ:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    use_gpu = torch.cuda.is_available() and not a.cpu
    # captured by default: at world size > 1 for the collective overlap; at world size 1 the
    # toy MLP's eager step is bound by host-side launch work (r6j: eager 0.375-0.47 ms, captured
    # 0.371-0.374 ms, profiles/r6/bench_modes_r6j.txt) and the CNN steps measured faster
    # captured on two boxes (ResNet-50 -0.4 / -0.6 %, AlexNet -2.0 %: profiles/r10/bench/r10s_*,
    # r10t_*); --eager for the eager step
    graph = use_gpu and not a.eager and a.impl == "tdp"
    in_shape = (dims[0],) if a.model == "toy_mlp" else (3, a.image_size, a.image_size)
    fused = False
    fallbacks = []
    rung = None
    job = None

    if a.impl == "tdp":
        import types

        import tutorial_torch_distributed_data_parallel_amd as tdp
        from tutorial_torch_distributed_data_parallel_amd.parallel import runtime as rt

        if a.comm_cus is not None and use_gpu:
            from tutorial_torch_distributed_data_parallel_amd._native import native as _nat

            _nat().set_reserved_cus(a.comm_cus)
        tdp.init_process_group("nccl" if use_gpu else "gloo")
        rank, world, dev = rt.get_rank(), rt.get_world_size(), rt.device()
        barrier = rt.barrier
        finish = tdp.destroy_process_group
        ctx = types.SimpleNamespace(dims=dims, in_shape=in_shape, use_gpu=use_gpu, rank=rank,
                                    world=world, dev=dev, graph=graph)
        fault = BenchFault()
    else:
        import torch.distributed as dist
        import torch.nn as nn
        from torch.nn.parallel import DistributedDataParallel as TorchDDP
        from torch.utils.data import DistributedSampler as TorchSampler

        rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if use_gpu:
            torch.cuda.set_device(local)
            dev = torch.device("cuda", local)
        else:
            dev = torch.device("cpu")
        if world > 1 or "MASTER_ADDR" in os.environ:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29511")
            dist.init_process_group("nccl" if use_gpu else "gloo", rank=rank, world_size=world)
        else:
            os.environ["MASTER_ADDR"] = "127.0.0.1"
            os.environ["MASTER_PORT"] = str(29600 + os.getpid() % 300)
            dist.init_process_group("nccl" if use_gpu else "gloo", rank=0, world_size=1)
        torch.manual_seed(1234 + rank)
        sys.path.insert(0, str(ROOT / "scripts"))
        from stock_models import stock_model

        model = stock_model(a.model, a.syncbn, dims=dims).to(dev)
        ddp = TorchDDP(model, device_ids=[local] if use_gpu else None,
                       bucket_cap_mb=a.bucket_mb if a.bucket_mb else 25)
        crit = nn.CrossEntropyLoss()
        opt = (torch.optim.SGD(ddp.parameters(), lr=0.01, momentum=0.9) if a.optim == "sgd"
               else torch.optim.Adam(ddp.parameters(), lr=1e-3))
        g = torch.Generator(device=dev)
        g.manual_seed(rank)
        X = torch.randn(a.dataset, *in_shape, generator=g, device=dev)
        Y = torch.randint(0, 10, (a.dataset,), generator=g, device=dev)

        class _DS:
            def __len__(self):
                return a.dataset
        sampler = TorchSampler(_DS(), num_replicas=world, rank=rank, shuffle=True)

        class _Loader:
            # same data path as the native bench: the epoch's indices go to the device once
            def __iter__(self):
                idx = torch.as_tensor(list(sampler), dtype=torch.long).to(dev)
                for s in range(0, len(idx) - len(idx) % a.batch, a.batch):
                    b = idx[s:s + a.batch]
                    yield X.index_select(0, b), Y.index_select(0, b)
        loader = _Loader()

        def barrier():
            dist.barrier()

        def finish():
            dist.destroy_process_group()

        def run_step(x, y):
            opt.zero_grad(set_to_none=True)
            loss = crit(ddp(x), y)
            loss.backward()
            opt.step()
            return loss

    sync = (torch.cuda.synchronize if use_gpu else (lambda: None))
    build_rehearsal = None
    if a.impl != "tdp":
        epoch = [0]
        it = [iter(loader)]

        def next_batch():
            try:
                return next(it[0])
            except StopIteration:
                epoch[0] += 1
                sampler.set_epoch(epoch[0])
                it[0] = iter(loader)
                return next(it[0])

        def step():
            return run_step(*next_batch())

    def clock_warmup():
        if use_gpu:
            mode = a.warmup_mode if a.warmup_mode != "auto" else \
                ("scratch" if a.model == "toy_mlp" else "gemm")
            if a.impl == "tdp" and mode == "scratch":
                scratch_warmup(a, dims, in_shape, dev)
            else:
                device_warmup(dev, a.device_warmup_ms, a.impl == "tdp")

    if a.impl == "tdp":
        # the fallback ladder (LADDER): build a rung, run its W warm-up steps; any failure on
        # any rank moves every rank to the next rung. World size 1 has no collectives to lose
        # and tries the full rung only, as before.
        import gc

        def timed_ms(j, n):
            """ms per step of n steps of job j, max over ranks (the selection's clock)."""
            barrier()
            sync()
            t0 = time.perf_counter()
            j.step.many(n)
            sync()
            barrier()
            t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64,
                             device=dev if use_gpu else "cpu")
            rt.all_reduce(t, "max")
            return float(t.item()) * 1000.0 / n

        def free_job():
            gc.collect()
            if use_gpu:
                torch.cuda.synchronize()
                torch.cuda.empty_cache()

        tensor_job, selection = None, None
        if world > 1 and a.parallel != "ddp" and a.model == "toy_mlp" and a.api == "ddp":
            # every tensor-sharded variant that builds is timed (same replay form as the timed
            # region: step.many); --parallel tensor measures the fastest, --parallel auto only
            # records their timings next to the DDP headline
            selection = {}
            for tcfg in TENSOR_RUNGS:
                ok, err, tj = True, None, None
                try:
                    tj = build_tdp(a, ctx, tcfg, 0, fallbacks, fault)
                    clock_warmup()
                    tj.step.many(a.warmup)
                    sync()
                except Exception as e:  # noqa: BLE001 - agreed below; the ladder follows
                    ok, err = False, e
                    _report_local(tcfg["name"], e)
                if not _agree(ok):
                    fallbacks.append(f"{tcfg['name']} failed ({repr(err)[:200] if err else 'on another rank'})")
                    print(f"[bench] {tcfg['name']} failed on some rank: {err!r}",
                          file=sys.stderr, flush=True)
                    tj = None
                else:
                    selection[f"{tcfg['name']}_ms"] = round(timed_ms(tj, a.select_steps), 4)
                    if a.parallel == "tensor" and (tensor_job is None or
                                                   selection[f"{tcfg['name']}_ms"] <
                                                   selection[f"{tensor_job.rung}_ms"]):
                        tensor_job = tj  # the previous best (if any) is released here
                    tj = None
                free_job()
        # --parallel auto / ddp: the headline is ALWAYS the DDP reducer's step (BASELINE metric
        # "toy-MLP DDP"); no tensor-sharded job survives into the ladder
        rungs = LADDER if world > 1 or os.environ.get("TDP_BENCH_LADDER") == "1" else LADDER[:1]
        if tensor_job is not None:
            rungs = ()
            job = tensor_job
            selection["chosen"] = job.rung
        elif selection is not None and a.parallel == "tensor":
            fallbacks.append("--parallel tensor: no tensor-sharded variant built; measured the "
                             "DDP ladder instead")
        for attempt, cfg in enumerate(rungs):
            ok, err = True, None
            try:
                job = build_tdp(a, ctx, cfg, attempt, fallbacks, fault)
                if attempt == 0:
                    clock_warmup()
                fault.check("warmup", attempt)
                job.step.many(a.warmup)
                sync()
            except Exception as e:  # noqa: BLE001 - agreed below, then the next rung
                ok, err = False, e
                _report_local(cfg["name"], e)
                if len(rungs) == 1:
                    raise
            if _agree(ok):
                break
            fallbacks.append(f"{cfg['name']} failed ({repr(err)[:200] if err else 'on another rank'})"
                             "; next rung")
            print(f"[bench] rung {cfg['name']} failed on some rank: {err!r}", file=sys.stderr,
                  flush=True)
            job = None
            free_job()
        else:
            if rungs:
                print("[bench] every rung of the fallback ladder failed: no timed step ran",
                      file=sys.stderr, flush=True)
                sys.exit(1)
        if selection is not None and job.tp is None:
            # auto: the DDP rung's own selection-form timing beside the tensor side numbers
            selection[f"{job.rung}_ms"] = round(timed_ms(job, a.select_steps), 4)
            selection["chosen"] = job.rung
        if selection is not None and job.tp is not None:
            # the chosen tensor job was timed before the other candidates were built: bring it
            # back to its warm state before the timed region
            job.step.many(a.warmup)
            sync()
        tensor_job = None
        ddp, opt, fused, step, run, graph = (job.ddp, job.opt, job.fused, job.step, job.run,
                                             job.graph)
        build_rehearsal, rung = job.build_rehearsal, job.rung
    else:
        clock_warmup()
        for _ in range(a.warmup):
            step()
    many = getattr(step, "many", None)
    barrier()
    sync()
    t0 = time.perf_counter()
    if many is not None:
        loss = many(a.steps)
    else:
        for _ in range(a.steps):
            loss = step()
    sync()
    barrier()
    sync()
    dt = time.perf_counter() - t0
    # max over ranks (the slowest rank defines the job's throughput)
    t = torch.tensor([dt], dtype=torch.float64, device=dev if use_gpu else "cpu")
    if world > 1:
        if a.impl == "tdp":
            rt.all_reduce(t, "max")
        else:
            import torch.distributed as dist
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    ms = dt * 1000.0 / a.steps
    value = a.batch * world * a.steps / dt
    base, base_src = baseline_for(world, a.impl, a.syncbn, a.model)
    final_loss = round(float(loss.item()), 5)
    sync = None
    if a.impl == "tdp" and ddp is not None:
        # self-report for the multi-GPU record: did every rank end with bit-identical
        # parameters, did the step run as a captured graph, how was each gradient synchronised
        from tutorial_torch_distributed_data_parallel_amd.train.graph import CapturedStep

        try:
            ddp.check_replicas()
            ident = True
        except RuntimeError:
            ident = False
        sync = {"replicas_identical": ident, "captured": isinstance(run, CapturedStep),
                "backend": rt.get_backend(), "modes": ddp.sync_plan(),
                "factor": ddp.factor_report() if ddp._factor else None,
                "factor_tuning": ddp.factor_tuning}

    if a.impl == "tdp" and getattr(job, "tp", None) is not None:
        from tutorial_torch_distributed_data_parallel_amd.train.graph import CapturedStep

        try:
            job.tp.check_replicas()
            ident = True
        except RuntimeError:
            ident = False
        sync = {"replicas_identical": ident, "captured": isinstance(run, CapturedStep),
                "backend": rt.get_backend(),
                "modes": {"fc1": "column-sharded", "fc2": "row-sharded (reduce-scatter of "
                          "activations)", "head": "replicated (averaged all-reduce)"}}
    comm_nranks = None
    if a.impl == "tdp" and rt.comm() is not None:
        comm_nranks = int(rt.comm().nranks)

    sel_ms = sel_warn = None
    if a.impl == "tdp" and selection and f"{rung}_ms" in selection:
        sel_ms = selection[f"{rung}_ms"]
        if abs(sel_ms - ms) > 0.2 * ms:
            sel_warn = (f"the selection clock ({sel_ms:.4f} ms) and the timed region "
                        f"({ms:.4f} ms) differ by more than 20 %")
            print(f"[bench] warning: {sel_warn}", file=sys.stderr, flush=True)

    def record(diag):
        desc = MODEL_DESC[a.model].format(s=a.image_size, dims="-".join(map(str, dims + (10,))),
                                          bn=", +SyncBatchNorm" if a.syncbn else "")
        tensor = a.impl == "tdp" and getattr(job, "tp", None) is not None
        if tensor:
            # not DDP: Megatron-style column/row-sharded fc1/fc2 (parallel/tensor_parallel.py),
            # labelled tp{N} so it is never read as the DDP headline
            impl = ("tdp tensor-sharded execution (column-parallel fc1, row-parallel fc2, "
                    f"replicated head; execution '{rung}'" +
                    (", hipGraph step)" if graph else ", eager)"))
        elif a.impl == "tdp":
            impl = "tdp (native gfx950 kernels + RCCL reducer" + \
                (", hipGraph step)" if graph else ", eager)")
            if a.api == "accelerate":
                impl += " via Accelerator.prepare()"
        else:
            impl = "stock torch DDP + torch.optim"
        rec = {
            "metric": metric if not tensor else
            "samples/sec (whole node) toy-MLP tensor-sharded (not DDP) at N MI355X",
            "value": round(value, 2),
            "unit": "samples/s",
            "n_gpus": world if use_gpu else 0,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / base, 4) if base else None,
            "dtype": "fp32",
            "data": "synthetic (on-device random features, random-init weights)",
            "config": {
                "model": desc,
                "global_batch": a.batch * world,
                "seq_len": None,
                "parallelism": f"{'tp' if tensor else 'dp'}{world}",
                "impl": impl,
                "optimizer": a.optim + ((" (shards: fused into their weight-gradient GEMMs)"
                                         if job.tp is not None else
                                         " (fused into the gradient reduction)")
                                        if a.impl == "tdp" and fused else ""),
                "final_loss": final_loss,
                # the toy MLP's head Linear + cross-entropy: one fused op or the two calls
                "head_loss": a.head_loss if a.model == "toy_mlp" and a.impl == "tdp" else None,
                "tp_data": ("replicated dataset, node batch gathered locally"
                            if a.tp_replicated_data else "per-rank batches, inputs all-gathered")
                if tensor else None,
                "device_warmup_ms": a.device_warmup_ms if use_gpu else 0,
                "comm_cus": _reserved_cus(a.impl, use_gpu),
                "bucket_mb": [round((ddp._bounds[i + 1] - ddp._bounds[i]) * 4 / 2 ** 20, 2)
                              for i in range(len(ddp._bounds) - 1)]
                if a.impl == "tdp" and ddp is not None else None,
                "gemm_products": _gemm_products(a.impl, use_gpu),
                "sync": sync,
                "launched_by": launched_by(),
                "comm_nranks": comm_nranks,
                # training steps per hipGraph replay (0: eager)
                "graph_steps": getattr(step, "graph_steps", None),
                # the fallback ladder (LADDER): the rung that ran and what failed before it
                "rung": rung,
                "fallbacks": fallbacks,
                # --parallel tensor / auto at N > 1: ms/step of each candidate (same replay
                # form as the timed region) and the one measured (auto: always the DDP rung)
                "selection": selection if a.impl == "tdp" else None,
                "selection_ms": sel_ms,
                "selection_gap_warning": sel_warn,
                "baseline": {"samples_per_s": round(base, 2), "source": base_src}
                if base else None,
            },
        }
        if diag is not None:
            rec["diagnostics"] = diag
        return rec

    diag = None
    tp_job = job if (a.impl == "tdp" and getattr(job, "tp", None) is not None) else None
    if tp_job is not None and use_gpu and not a.no_diag:
        limit = float(os.environ.get("TDP_DIAG_TIMEOUT_S", "120"))

        def expire_tp():
            if rank == 0:
                print(json.dumps(record({"error": f"diagnostics exceeded {limit:g} s"})),
                      file=out, flush=True)
            os._exit(0)
        timer = threading.Timer(limit, expire_tp)
        timer.daemon = True
        timer.start()
        try:
            diag = tensor_diagnostics(a, tp_job, ms, world, barrier)
        except Exception as e:  # diagnostics never cost the measurement
            diag = {"error": repr(e)[:300]}
        timer.cancel()
    if a.impl == "tdp" and ddp is not None and use_gpu and not a.no_diag:
        # The measurement is final here. Diagnostics run more collectives, and a peer that
        # stalls in them must not cost the result: past the deadline every rank exits 0, and
        # rank 0 first prints the record without them.
        limit = float(os.environ.get("TDP_DIAG_TIMEOUT_S", "120"))

        def expire():
            if rank == 0:
                print(json.dumps(record({"error": f"diagnostics exceeded {limit:g} s"})),
                      file=out, flush=True)
            os._exit(0)
        timer = threading.Timer(limit, expire)
        timer.daemon = True
        timer.start()
        try:
            diag = diagnostics(a, ddp, step, ms, world, graph, barrier, build_rehearsal)
        except Exception as e:  # diagnostics never cost the measurement
            diag = {"error": repr(e)[:300]}
        timer.cancel()
    if rank == 0:
        print(json.dumps(record(diag)), file=out, flush=True)
    finish()


if __name__ == "__main__":
    main()
