"""Step model of the gradient synchronisation of a Linear stack at W ranks (SURVEY.md §5.8;
VERDICT r3 item 3: "publish the model ... per-rank bytes and predicted exposed us at W=2/4/8").

Two timelines of one captured step are simulated: the compute stream (forward, then backward
layer by layer) and the communicator's side stream, which runs the sync jobs in issue order.
Each Linear weight W[out][in] (per-rank batch B) is synchronised in one of four modes:

  allreduce           ring all-reduce of the out*in gradient, update on every rank
  sharded             reduce-scatter -> update own 1/W -> all-gather of the parameters
                      (same wire bytes as allreduce, 1/W of the optimizer traffic)
  factored-sharded    all-gather the factors g [B][out] and x [B][in] (x at FORWARD time,
                      ops/linear.py -> DDP.factor_forward), GEMM of depth W*B for this rank's
                      out/W rows with the update in its epilogue, all-gather of the rows
  factored-replicated the same gathers, the GEMM over ALL rows on every rank, no parameter
                      all-gather

A job can start when its gradient factor exists (backward of the layer above) and when the
side stream is free; the step ends when both streams are done, so the exposed communication is
``max(0, side_end - compute_end)``. Wire times use bus bandwidth (nccl-tests convention):
``t = bytes * factor / busbw`` with factor 2(W-1)/W (all-reduce) or (W-1)/W (all-gather,
reduce-scatter), plus a fixed latency per collective. Compute on the side stream (the factored
GEMM, updates) is costed at the given rates and assumed not to slow the compute stream -- an
optimistic bound, stated as such in docs/COMM_MODEL.md.

Inputs are either assumed (``Hardware``: per-link xGMI bandwidth x links used, the split-bf16
fp32 GEMM rate, HBM bandwidth) or measured (bench.py passes the RCCL busbw of its diagnostic
sweep). Layer compute times default to the dp1 kernel table of the toy MLP
(profiles/r7/mlp_kernels_r7e_final.md) and scale with FLOPs for other shapes.
"""
from __future__ import annotations

from dataclasses import dataclass, field

MODES = ("allreduce", "sharded", "factored-sharded", "factored-replicated")


@dataclass
class Hardware:
    link_GBps: float = 51.0        # effective unidirectional GB/s per xGMI link (64 peak x 0.8)
    gemm_TFps: float = 170.0       # split-bf16 fp32 GEMM (profiles/micro: 168-170 TF/s at 4096^3)
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
    """Per-rank wire bytes and side-stream time (us) of one weight's sync job. ``x_us`` is the
    part issued at forward time (factored x gather), the rest runs when g is ready."""
    o, n = layer.out, layer.inp
    P = 4.0 * o * n
    upd_full = 16.0 * o * n / (hw.hbm_TBps * 1e6)     # p + momentum read + write (SGD)
    if mode == "allreduce":
        t = _coll_us(hw, "all_reduce", W, P) + upd_full
        return {"mode": mode, "wire_MB": 2 * (W - 1) / W * P / 1e6, "x_us": 0.0, "g_us": t,
                "compute_wgrad_us": layer.wgrad_us - 0.0}
    if mode == "sharded":
        t = _coll_us(hw, "reduce_scatter", W, P) + upd_full / W + _coll_us(hw, "all_gather", W, P)
        return {"mode": mode, "wire_MB": 2 * (W - 1) / W * P / 1e6, "x_us": 0.0, "g_us": t,
                "compute_wgrad_us": layer.wgrad_us}
    gx = 4.0 * B * n * W               # gathered x bytes (W slots)
    gg = 4.0 * B * o * W
    x_us = _coll_us(hw, "all_gather", W, gx)
    g_us = _coll_us(hw, "all_gather", W, gg)
    rows = o if mode == "factored-replicated" else o / W
    gemm = 2.0 * W * B * rows * n / (hw.gemm_TFps * 1e6)
    upd = 16.0 * rows * n / (hw.hbm_TBps * 1e6)
    t = g_us + max(gemm, upd)
    wire = (gx + gg) * (W - 1) / W
    if mode == "factored-sharded":
        t += _coll_us(hw, "all_gather", W, P)
        wire += P * (W - 1) / W
    return {"mode": mode, "wire_MB": wire / 1e6, "x_us": x_us, "g_us": t,
            "compute_wgrad_us": 0.0}


def simulate(layers: list[Layer], modes: dict, W: int, B: int, hw: Hardware,
             prefetch_x: bool = True) -> dict:
    """Predicted step of a captured W-rank step: compute-stream time, side-stream end, exposed
    communication and the per-job table. ``modes``: layer name -> mode (layers absent, e.g. the
    small head, ride in the first bucket: all-reduced with the job of the layer below them)."""
    t = 0.0
    side = 0.0
    jobs = []
    costs = {L.name: job_cost(L, modes[L.name], W, B, hw) for L in layers if L.name in modes}
    # forward: the factored layers' x gathers start as soon as the layer runs
    for L in layers:
        t += L.fwd_us
        c = costs.get(L.name)
        if c and c["x_us"] > 0 and prefetch_x:
            start = max(side, t - L.fwd_us)
            side = start + c["x_us"]
    fwd_end = t
    # backward, last layer first: a layer's job starts once its g exists (after the layer
    # above's input gradient); its own dgrad / wgrad run on the compute stream
    small = [L for L in layers if L.name not in modes]
    t += sum(L.dgrad_us + L.wgrad_us for L in small)
    # small layers' gradients ride with the next job: an all-reduce of their bytes
    small_bytes = sum(4.0 * L.out * L.inp for L in small)
    for L in reversed([L for L in layers if L.name in modes]):
        c = costs[L.name]
        ready = t
        start = max(side, ready)
        dur = c["g_us"] + (0.0 if prefetch_x else c["x_us"])
        if small_bytes:
            dur += _coll_us(hw, "all_reduce", W, small_bytes)
            small_bytes = 0.0
        side = start + dur
        jobs.append({"layer": L.name, **{k: round(v, 2) if isinstance(v, float) else v
                                         for k, v in c.items()},
                     "start_us": round(start, 1), "end_us": round(side, 1)})
        t += L.dgrad_us + c["compute_wgrad_us"]
    exposed = max(0.0, side - t)
    return {"W": W, "B": B, "compute_us": round(t, 1), "forward_us": round(fwd_end, 1),
            "side_end_us": round(side, 1), "exposed_us": round(exposed, 1),
            "step_us": round(max(t, side), 1), "jobs": jobs}


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
