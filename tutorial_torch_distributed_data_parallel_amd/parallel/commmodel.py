"""Step model of the gradient synchronisation of a Linear stack at W ranks (SURVEY.md §5.8;
VERDICT r3 item 3: "publish the model ... per-rank bytes and predicted exposed us at W=2/4/8").

Two timelines of one captured step are simulated: the compute stream (forward, then backward
layer by layer, plus the sync jobs' arithmetic) and the communicator's side stream, which runs
the collectives in issue order.
Each Linear weight W[out][in] (per-rank batch B) is synchronised in one of four modes:

  allreduce           ring all-reduce of the out*in gradient, update on every rank
  sharded             reduce-scatter -> update own 1/W -> all-gather of the parameters
                      (same wire bytes as allreduce, 1/W of the optimizer traffic)
  factored-sharded    all-gather the factors g [B][out] and x [B][in] (x at FORWARD time,
                      ops/linear.py -> DDP.factor_forward), GEMM of depth W*B for this rank's
                      out/W rows with the update in its epilogue, all-gather of the rows
  factored-replicated the same gathers, the GEMM over ALL rows on every rank, no parameter
                      all-gather
  factored-split      a fraction f of the rows replicated, the rest sharded: this rank's shard
                      GEMM first, then the all-gather of the sharded rows on the side stream
                      WHILE the compute stream computes the replicated rows (f balances the two)

A job's collectives start when its gradient factor exists (backward of the layer above) and
the side stream is free; its arithmetic runs on the compute stream once they are in; the step
ends when both streams are done, so the exposed communication is the step minus the compute a
single rank would do. Wire times use bus bandwidth (nccl-tests convention):
``t = bytes * factor / busbw`` with factor 2(W-1)/W (all-reduce) or (W-1)/W (all-gather,
reduce-scatter), plus a fixed latency per collective. Compute on the side stream (the factored
GEMM, updates) is costed at the given rates; collectives are assumed not to slow the compute
kernels they overlap -- an optimistic bound, stated as such in docs/COMM_MODEL.md.

Inputs are either assumed (``Hardware``: per-link xGMI bandwidth x links used, the split-bf16
fp32 GEMM rate, HBM bandwidth) or measured (bench.py passes the RCCL busbw of its diagnostic
sweep). Layer compute times default to the dp1 kernel table of the toy MLP
(profiles/r7/mlp_kernels_r7e_final.md) and scale with FLOPs for other shapes.
"""
from __future__ import annotations

from dataclasses import dataclass, field

MODES = ("allreduce", "sharded", "factored-sharded", "factored-replicated", "factored-split")


@dataclass
class Hardware:
    link_GBps: float = 51.0        # effective unidirectional GB/s per xGMI link (64 peak x 0.8)
    # split-bf16 fp32 GEMM with the optimizer epilogue, the kernel a factored job runs
    # (gemm_f32_fast: 175.2 TF/s at 4096 x 4096 x 9216, profiles/r9/gemm_emu8_r9.md; the
    # 205 TF/s 256 x 256 kernel of that table has no optimizer epilogue and is not dispatched
    # for these jobs)
    gemm_TFps: float = 175.0
    hbm_TBps: float = 5.0          # optimizer streams (profiles/r7: 4.3-4.5 in the epilogue)
    latency_us: float = 12.0       # per collective launch + sync on xGMI
    busbw_GBps: dict = field(default_factory=dict)  # measured: {"all_gather": x, ...} overrides

    def busbw(self, op: str, W: int) -> float:
        if op in self.busbw_GBps:
            return float(self.busbw_GBps[op])
        # a full mesh: W-1 direct links per rank carry the traffic of a direct / multi-ring
        # algorithm; a 2-rank job has one link
        return self.link_GBps * max(1, W - 1)


@dataclass
class Layer:
    name: str
    out: int
    inp: int
    fwd_us: float      # forward GEMM (+ epilogue)
    dgrad_us: float    # input-gradient GEMM (0 for the first layer)
    wgrad_us: float    # weight-gradient GEMM with the update in its epilogue (dp1)


def toy_mlp_layers(B: int = 128, dims=(9216, 4096, 4096), classes: int = 10) -> list[Layer]:
    """The headline model with the dp1 kernel times of profiles/r7/mlp_kernels_r7e_final.md
    (B=128), scaled by FLOPs for other shapes."""
    d0, d1, d2 = dims
    s = B / 128.0
    f1 = 2.0 * d0 * d1 / (2.0 * 9216 * 4096)
    f2 = 2.0 * d1 * d2 / (2.0 * 4096 * 4096)
    return [Layer("fc1", d1, d0, 58.7 * f1 * s, 0.0, 135.4 * f1 * s),
            Layer("fc2", d2, d1, 30.1 * f2 * s, 30.1 * f2 * s, 65.4 * f2 * s),
            Layer("fc3", classes, d2, 6.0, 7.8, 0.0)]


def _coll_us(hw: Hardware, op: str, W: int, nbytes: float) -> float:
    if W <= 1 or nbytes <= 0:
        return 0.0
    factor = 2.0 * (W - 1) / W if op == "all_reduce" else (W - 1) / W
    return hw.latency_us + nbytes * factor / (hw.busbw(op, W) * 1e3)


def job_cost(layer: Layer, mode: str, W: int, B: int, hw: Hardware) -> dict:
    """Per-rank wire bytes and the parts of one weight's sync job, in us: ``x_us`` the factored
    x gather (issued at forward time), ``pre_us`` side-stream collectives before the update
    arithmetic, ``compute_us`` the arithmetic (wgrad GEMM / factored GEMM + update; on the
    compute stream), ``post_us`` side-stream collectives after it. ``g_us`` = pre + compute +
    post: the job alone, serialised."""
    o, n = layer.out, layer.inp
    P = 4.0 * o * n
    # bucket modes: the weight-gradient GEMM and one update pass (layer.wgrad_us: the dp1
    # epilogue GEMM, which does both) on the compute stream, the collectives on the side stream
    if mode == "allreduce":
        pre, comp, post = 0.0, layer.wgrad_us, _coll_us(hw, "all_reduce", W, P)
        wire = 2 * (W - 1) / W * P
        x_us = 0.0
    elif mode == "sharded":
        pre, comp = 0.0, layer.wgrad_us
        post = _coll_us(hw, "reduce_scatter", W, P) + _coll_us(hw, "all_gather", W, P)
        wire = 2 * (W - 1) / W * P
        x_us = 0.0
    else:
        gx = 4.0 * B * n * W               # gathered x bytes (W slots)
        gg = 4.0 * B * o * W
        x_us = _coll_us(hw, "all_gather", W, gx)
        pre = _coll_us(hw, "all_gather", W, gg)

        def arith(rows):
            gemm = 2.0 * W * B * rows * n / (hw.gemm_TFps * 1e6)
            return max(gemm, 16.0 * rows * n / (hw.hbm_TBps * 1e6))
        f = 1.0 if mode == "factored-replicated" else 0.0
        if mode == "factored-split" and W > 1:
            # balance the replicated rows' arithmetic against the all-gather of the others
            ag = _coll_us(hw, "all_gather", W, P)
            f = max(0.0, min(1.0, ag / (ag + arith(o))))
        comp = arith(o * f) if mode == "factored-replicated" else arith((1.0 - f) * o / W)
        after = arith(o * f) if mode == "factored-split" else 0.0
        post = 0.0 if mode == "factored-replicated" else \
            _coll_us(hw, "all_gather", W, (1.0 - f) * P)
        wire = (gx + gg) * (W - 1) / W + (1.0 - f) * P * (W - 1) / W * (mode != "factored-replicated")
        return {"mode": mode, "wire_MB": wire / 1e6, "x_us": x_us, "pre_us": pre,
                "compute_us": comp, "after_us": after, "post_us": post, "rep_fraction": f,
                "g_us": pre + comp + max(post, after)}
    return {"mode": mode, "wire_MB": wire / 1e6, "x_us": x_us, "pre_us": pre,
            "compute_us": comp, "after_us": 0.0, "post_us": post, "rep_fraction": 0.0,
            "g_us": pre + comp + post}


def simulate(layers: list[Layer], modes: dict, W: int, B: int, hw: Hardware,
             prefetch_x: bool = True, early_g: bool = True) -> dict:
    """Predicted captured W-rank step (reducer.cpp / ops/linear.py schedule): forward issues the
    factored x gathers on the side stream; backward runs, per weight from the last layer down,
    the layer's input gradient and then its job -- side-stream collectives (gathers, all-reduce,
    parameter all-gather) in FIFO order, the job's arithmetic on the compute stream once its
    gathers are in. A factored layer's g gather goes out before its input-gradient GEMM, or with
    ``early_g`` one layer earlier: right after the consumer's (gated) input-gradient GEMM, which
    produces that g, so it precedes the consumer's parameter all-gather in the FIFO. The step
    ends when both streams are done: ``exposed_us`` = step - compute alone. ``modes``: layer
    name -> mode; layers absent (the small head) cost their compute time and ride, as an
    all-reduce, with the first job."""
    tc = ts = 0.0
    costs = {L.name: job_cost(L, modes[L.name], W, B, hw) for L in layers if L.name in modes}
    for L in layers:  # forward
        if L.name in costs and costs[L.name]["x_us"] > 0 and prefetch_x:
            ts = max(ts, tc) + costs[L.name]["x_us"]
        tc += L.fwd_us
    fwd_end = tc
    alone = fwd_end + sum(L.dgrad_us + L.wgrad_us for L in layers)  # dp1-like compute
    small = [L for L in layers if L.name not in modes]
    tc += sum(L.dgrad_us + L.wgrad_us for L in small)
    small_bytes = sum(4.0 * L.out * L.inp for L in small)
    jobs = []
    order = list(reversed([L for L in layers if L.name in modes]))
    gathered = {}  # layer -> (start, end) of its pre-job collectives on the side stream

    def pre_of(L):
        nonlocal small_bytes
        pre = costs[L.name]["pre_us"] + (0.0 if prefetch_x else costs[L.name]["x_us"])
        if small_bytes:
            pre += _coll_us(hw, "all_reduce", W, small_bytes)
            small_bytes = 0.0
        return pre

    for k, L in enumerate(order):
        c = costs[L.name]
        if L.name not in gathered:       # its g exists now: gathered before its dgrad
            start = max(ts, tc)
            ts = start + pre_of(L)
            gathered[L.name] = (start, ts)
        tc += L.dgrad_us                 # its input gradient (captured before the job's fork)
        nxt = order[k + 1] if k + 1 < len(order) else None
        if early_g and nxt is not None and costs[nxt.name]["mode"].startswith("factored"):
            start = max(ts, tc)          # the gated dx is nxt's g
            ts = start + pre_of(nxt)
            gathered[nxt.name] = (start, ts)
        start, done = gathered[L.name]
        tc = max(tc, done if c["mode"].startswith("factored") else tc) + c["compute_us"]
        if c["post_us"] > 0:
            ts = max(ts, tc) + c["post_us"]
        tc += c["after_us"]  # replicated rows of a split job, while its all-gather runs
        jobs.append({"layer": L.name, **{k2: round(v, 2) if isinstance(v, float) else v
                                         for k2, v in c.items()},
                     "start_us": round(start, 1), "end_us": round(max(ts, tc), 1)})
    step = max(tc, ts)
    return {"W": W, "B": B, "compute_us": round(alone, 1), "forward_us": round(fwd_end, 1),
            "side_end_us": round(ts, 1), "exposed_us": round(max(0.0, step - alone), 1),
            "step_us": round(step, 1), "jobs": jobs}


# Per-rank compute of the tensor-sharded step (parallel/tensor_parallel.py), measured on one GPU
# with the shard shapes of W ranks and the collectives replaced by local copies
# (scripts/tp_rank_proxy.py, profiles/r9/tp_rank_proxy_fused_r9ak.jsonl: the shards' SGD in their
# weight-gradient GEMM epilogues, TensorParallelMLP.register_fused_optimizer; dp1 of that run:
# 349.8 us. Before the fused update, r9x: 371.0 / 360.4 / 354.6 against dp1 357.6)
TP_RANK_US = {1: 490.0, 2: 341.8, 4: 331.3, 8: 339.4}
TP_DP1_US = 349.8


def simulate_tensor(W: int, B: int = 128, dims=(9216, 4096, 4096), classes: int = 10,
                    hw: Hardware | None = None, chunks: int = 1, global_batch: bool = True,
                    rank_us: float | None = None, fc2_gemm_us: float = 42.0) -> dict:
    """Predicted step of the tensor-sharded toy MLP at W ranks: the measured per-rank compute
    plus the collectives on its critical path -- the reduce-scatter of fc2's partial output
    [W*B, h2] (forward) and the all-gather of its gradient (backward), the averaged all-reduce
    of the replicated head, and (without ``global_batch``) the input all-gather. With ``chunks``
    > 1 each of the two big collectives runs in column chunks behind fc2's chunk GEMMs
    (``fc2_gemm_us``: that layer's forward GEMM time, the backward has two such GEMMs)."""
    hw = hw or Hardware()
    d0, h1, h2 = dims
    if W <= 1:
        c = rank_us if rank_us is not None else TP_RANK_US.get(1, TP_DP1_US)
        return {"W": 1, "compute_us": c, "exposed_us": 0.0, "step_us": c, "wire_MB": 0.0}
    comp = rank_us if rank_us is not None else TP_RANK_US.get(W, TP_RANK_US[8])
    big = 4.0 * W * B * h2
    rs = _coll_us(hw, "reduce_scatter", W, big)
    ag = _coll_us(hw, "all_gather", W, big)
    head = _coll_us(hw, "all_reduce", W, 4.0 * (h2 * classes + classes + h2))
    xg = 0.0 if global_batch else _coll_us(hw, "all_gather", W, 4.0 * W * B * d0)

    def hidden(coll, gemm):
        """Exposed part of a collective split into ``chunks`` behind as many GEMM chunks."""
        if chunks <= 1:
            return coll
        g, c = gemm / chunks, (coll - hw.latency_us) / chunks + hw.latency_us
        return g + (chunks - 1) * max(g, c) + c - gemm

    # the head's all-reduce is issued on the communication stream right after the backward
    # all-gather and runs behind fc2's / fc1's gradient GEMMs (~4 x fc2_gemm_us of work)
    exposed = hidden(rs, fc2_gemm_us) + hidden(ag, 2 * fc2_gemm_us) + \
        max(0.0, head - 4 * fc2_gemm_us) + xg
    wire = (W - 1) / W * (2 * big + (0 if global_batch else 4.0 * W * B * d0)) + \
        2 * (W - 1) / W * 4.0 * (h2 * classes + classes + h2)
    return {"W": W, "compute_us": round(comp, 1), "exposed_us": round(exposed, 1),
            "step_us": round(comp + exposed, 1), "wire_MB": round(wire / 1e6, 1),
            "scaling_eff": round(TP_DP1_US / (comp + exposed), 3)}


def factored_bound(layers: list[Layer], W: int, B: int, hw: Hardware, steps: int = 40) -> dict:
    """Schedule-independent lower bound of the factored DDP step: whatever the order of jobs,
    forks and joins (including overlap ACROSS steps: the next forward waiting only for the
    parameters it reads), the compute stream must run the forward, the input gradients, the
    small layers and every job's arithmetic, and the links must carry every job's factor
    gathers plus the all-gather of its sharded rows. With a fraction f of a weight's rows
    replicated (0 = factored-sharded, 1 = factored-replicated) the step is at least
    max(compute(f), wire(f)); this minimises that over f per weight (grid of ``steps``). The
    achieved schedule (``simulate``) can only be slower."""
    import itertools

    big = [L for L in layers if L.out > 16]
    base = sum(L.fwd_us + L.dgrad_us for L in layers) + \
        sum(L.wgrad_us for L in layers if L not in big)
    small_bytes = sum(4.0 * L.out * L.inp for L in layers if L not in big)
    wire0 = _coll_us(hw, "all_reduce", W, small_bytes)

    def parts(L, f):
        o, n = L.out, L.inp

        def arith(rows):
            return max(2.0 * W * B * rows * n / (hw.gemm_TFps * 1e6),
                       16.0 * rows * n / (hw.hbm_TBps * 1e6))
        comp = arith(f * o) + arith((1.0 - f) * o / W)
        wire = _coll_us(hw, "all_gather", W, 4.0 * B * n * W) + \
            _coll_us(hw, "all_gather", W, 4.0 * B * o * W) + \
            (_coll_us(hw, "all_gather", W, (1.0 - f) * 4.0 * o * n) if f < 1.0 else 0.0)
        return comp, wire
    grid = [i / steps for i in range(steps + 1)]
    best = None
    for fs in itertools.product(grid, repeat=len(big)):
        c, w = base, wire0
        for L, f in zip(big, fs):
            dc, dw = parts(L, f)
            c += dc
            w += dw
        t = max(c, w)
        if best is None or t < best["step_us"]:
            best = {"step_us": round(t, 1), "compute_us": round(c, 1), "wire_us": round(w, 1),
                    "rep_fraction": {L.name: f for L, f in zip(big, fs)}}
    return best


def best_plan(layers: list[Layer], W: int, B: int, hw: Hardware,
              candidates: dict | None = None) -> dict:
    """The cheapest mode per weight (exhaustive over the candidates; the toy MLP has two)."""
    import itertools

    names = [L.name for L in layers if candidates is None or L.name in candidates]
    names = [n for n in names if any(L.name == n and L.out > 16 for L in layers)]
    best = None
    for combo in itertools.product(MODES, repeat=len(names)):
        modes = dict(zip(names, combo))
        if candidates:
            if any(m not in candidates[n] for n, m in modes.items()):
                continue
        r = simulate(layers, modes, W, B, hw)
        r["modes"] = modes
        if best is None or r["step_us"] < best["step_us"]:
            best = r
    return best


# ----------------------------------------------------------------------------- CNN buckets
# BASELINE config 5 ("ResNet-50-sized CNN DDP 8x: stresses grad-bucket all-reduce overlap"): the
# convolution weights are not factored (their gradient is not low-rank in a useful way), so they
# go through the bucket path -- per bucket a reduce-scatter, the 1/W optimizer update and the
# parameter all-gather on the side stream while backward continues (reducer.cpp SyncBackend).

# dp1 kernel times (ms per step, B = 128, 224 x 224) the per-layer backward times are scaled to:
# GEMM / convolution forward and backward, BatchNorm backward passes
# (profiles/resnet50_dp1_b128_r4e.md, profiles/alexnet_dp1_b128_r4e.md)
CNN_DP1_MS = {"resnet50": {"gemm": 23.5, "bn_bwd": 6.1, "fwd_other": 5.0},
              "alexnet": {"gemm": 4.0, "bn_bwd": 0.0, "fwd_other": 0.3}}


@dataclass
class Grad:
    name: str
    numel: int
    bwd_us: float      # backward compute that ends with this gradient ready (its layer's share)


def cnn_grads(model: str = "resnet50", image: int = 224, times: dict | None = None):
    """(forward us, [Grad] in backward order) for a tdp CNN (models/registry.py): the module
    order of one forward (hooks), per-layer backward time in proportion to 2 x its forward FLOPs
    (convolutions / Linear: input + weight gradient) or to its output size (BatchNorm), scaled to
    the model's measured dp1 kernel times (CNN_DP1_MS). Runs a B = 1 forward on the CPU."""
    import torch

    from .. import nn as tnn
    from ..models.registry import build_model

    t = dict(CNN_DP1_MS[model], **(times or {}))
    m = build_model(model, device="cpu")
    rec = []

    def hook(mod, inp, out):
        w = getattr(mod, "weight", None)
        if isinstance(mod, (tnn.Conv2d, tnn.Linear)):
            flops = 2.0 * out.numel() * (w.numel() // w.shape[0])
            rec.append((mod, "gemm", flops))
        else:
            rec.append((mod, "bn", float(out.numel())))
    for mod in m.modules():
        if isinstance(mod, (tnn.Conv2d, tnn.Linear)) or "BatchNorm" in type(mod).__name__:
            mod.register_forward_hook(hook)
            if hasattr(mod, "relu_join"):  # bn3's fused residual join bypasses forward()
                def joined(*args, _f=mod.relu_join, _m=mod, **kw):
                    y = _f(*args, **kw)
                    hook(_m, args, y)
                    return y
                mod.relu_join = joined
    with torch.no_grad():
        m(torch.randn(1, 3, image, image))
    gemm_tot = sum(c for _, k, c in rec if k == "gemm") or 1.0
    bn_tot = sum(c for _, k, c in rec if k == "bn") or 1.0
    # forward = a third of the GEMM time + the rest of the forward passes; backward = the other
    # two thirds + the BN backward passes
    fwd_us = 1e3 * (t["gemm"] / 3.0 + t["fwd_other"])
    names = {id(p): n for n, p in m.named_parameters()}
    out = []
    for mod, kind, c in reversed(rec):
        us = 1e3 * (2.0 * t["gemm"] / 3.0 * c / gemm_tot if kind == "gemm"
                    else t["bn_bwd"] * c / bn_tot)
        ps = [p for p in (getattr(mod, "bias", None), getattr(mod, "weight", None))
              if isinstance(p, torch.nn.Parameter)]
        for j, p in enumerate(ps):  # the layer's time ends with its last gradient
            out.append(Grad(names[id(p)], p.numel(), us if j == len(ps) - 1 else 0.0))
    return fwd_us, out


def simulate_buckets(fwd_us: float, grads: list, W: int, hw: Hardware, first_mb: float = 1.0,
                     cap_mb: float = 25.0, mode: str = "sharded") -> dict:
    """Predicted captured CNN step at W ranks with the bucket plan (first bucket ``first_mb``,
    then ``cap_mb``; reducer.cpp compute_bucket_bounds): each bucket's collectives (``sharded``:
    reduce-scatter + all-gather around the 1/W update; ``allreduce``: one all-reduce + the full
    update) start on the side stream once its last gradient is ready and the side stream is
    free. ``exposed_us`` = step - (forward + backward + the one-rank update)."""
    buckets, cur, cur_b, lim = [], [], 0.0, first_mb
    for g in grads:
        cur.append(g)
        cur_b += 4.0 * g.numel
        if cur_b >= lim * 2 ** 20:
            buckets.append(cur)
            cur, cur_b, lim = [], 0.0, cap_mb
    if cur:
        buckets.append(cur)
    tc, ts = fwd_us, 0.0
    upd_alone = 16.0 * sum(g.numel for g in grads) / (hw.hbm_TBps * 1e6)
    for bk in buckets:
        tc += sum(g.bwd_us for g in bk)
        nbytes = 4.0 * sum(g.numel for g in bk)
        if mode == "allreduce":
            comm = _coll_us(hw, "all_reduce", W, nbytes)
            upd = 16.0 * nbytes / 4.0 / (hw.hbm_TBps * 1e6)
        else:
            comm = _coll_us(hw, "reduce_scatter", W, nbytes) + _coll_us(hw, "all_gather", W, nbytes)
            upd = 16.0 * nbytes / 4.0 / W / (hw.hbm_TBps * 1e6)
        ts = max(ts, tc) + comm + upd
    step = max(tc, ts)
    alone = tc + upd_alone
    return {"W": W, "buckets": len(buckets), "first_mb": first_mb, "cap_mb": cap_mb,
            "mode": mode, "compute_us": round(alone, 1), "step_us": round(step, 1),
            "exposed_us": round(max(0.0, step - alone), 1),
            "last_bucket_mb": round(4.0 * sum(g.numel for g in buckets[-1]) / 2 ** 20, 2)}


def table(W_list=(2, 4, 8), B: int = 128, hw: Hardware | None = None) -> list[dict]:
    """Rows for docs/COMM_MODEL.md: every uniform mode and the best per-weight plan per W."""
    hw = hw or Hardware()
    layers = toy_mlp_layers(B)
    big = [L.name for L in layers if L.out > 16]
    rows = []
    for W in W_list:
        for mode in MODES:
            r = simulate(layers, {n: mode for n in big}, W, B, hw)
            rows.append({"W": W, "plan": mode, "wire_MB": round(sum(j["wire_MB"] for j in r["jobs"]), 1),
                         "step_us": r["step_us"], "exposed_us": r["exposed_us"]})
        b = best_plan(layers, W, B, hw)
        rows.append({"W": W, "plan": "best: " + ", ".join(f"{k}={v}" for k, v in b["modes"].items()),
                     "wire_MB": round(sum(j["wire_MB"] for j in b["jobs"]), 1),
                     "step_us": b["step_us"], "exposed_us": b["exposed_us"]})
    return rows


if __name__ == "__main__":
    import json
    import sys

    for row in table():
        print(json.dumps(row))
    sys.exit(0)
