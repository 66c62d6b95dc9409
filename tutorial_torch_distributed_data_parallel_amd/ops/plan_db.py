"""Measured convolution GEMM plans (tile width FN, split-K) per exact geometry: a perf-db.

The planner in csrc/gemm_f32_fast.hip picks a plan from the GEMM shape alone. It cannot price wave
quantisation. A grid of T workgroups on 3 (FN 1) or 2 (FN 2) slots per CU runs ceil(T / slots)
rounds, so a near-empty last round can cost a fifth of the kernel. ResNet-50's layer3/4 3x3
convolutions are the measured case: 342 -> 286 us forward. `scripts/tune_conv_plans.py` measures
every (FN, split-K) per convolution and pass. It writes the winners that beat the heuristic by
>= 3 % to `perfdb/gfx950_conv_plans.json`. This module registers them with the native planner
(`conv_plan_db_put`), keyed by the exact NHWC GEMM geometry of each call, so the same table
serves eager and captured steps. A geometry missing from the table uses the heuristic.
(MIOpen's find-db / perf-db keeps tuned solver configs per problem in the same way.)
"""
from __future__ import annotations

import json
import os

_MODES = {"fwd": 0, "dgrad": 1, "wgrad": 2}
DEFAULT_DB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "perfdb",
                          "gfx950_conv_plans.json")
_loaded = False


def _out(n, k, s, p):
    return (n + 2 * p - k) // s + 1


def conv_geoms(mode: str, x_shape, w_shape, stride, padding):
    """The NHWC GEMM geometries `[N, C, H, W, Cout, R, S, P, Q, sh, sw, ph, pw]` one pass of a
    convolution launches (ops/conv.py): one for the forward / weight gradient / stride-1 input
    gradient, one per stride phase of a strided input gradient (`_dgrad_phases`)."""
    N, Cin, H, W = (int(v) for v in x_shape)
    Cout, _, R, S = (int(v) for v in w_shape)
    sh, sw = stride
    ph, pw = padding
    Cp = (Cin + 3) // 4 * 4
    P, Q = _out(H, R, sh, ph), _out(W, S, sw, pw)
    if mode != "dgrad" or (sh == 1 and sw == 1):
        return [[N, Cp, H, W, Cout, R, S, P, Q, sh, sw, ph, pw]]
    geoms = []
    for a in range(sh):
        r0 = (a + ph) % sh
        Rp, Hp, da = len(range(r0, R, sh)), len(range(a, H, sh)), (a + ph - r0) // sh
        for b in range(sw):
            s0 = (b + pw) % sw
            Sp, Wp, db = len(range(s0, S, sw)), len(range(b, W, sw)), (b + pw - s0) // sw
            if Hp and Wp and Rp and Sp:
                geoms.append([N, Cp, Hp, Wp, Cout, Rp, Sp, P, Q, 1, 1, da, db])
    return geoms


def register(C, entries) -> int:
    n = 0
    for e in entries:
        for g in conv_geoms(e["pass"], e["x"], e["w"], tuple(e["stride"]), tuple(e["padding"])):
            C.conv_plan_db_put(_MODES[e["pass"]], g, int(e["fn"]), int(e["splits"]))
            n += 1
    return n


def load(C, path: str = DEFAULT_DB) -> int:
    """Register a plan table (JSON list of entries); returns the geometries registered."""
    if not os.path.exists(path):
        return 0
    with open(path) as f:
        return register(C, json.load(f)["plans"])


def ensure_loaded(C) -> None:
    """Load the default table once per process (TDP_CONV_PLAN_DB=0 disables it; a path selects
    another table)."""
    global _loaded
    if _loaded:
        return
    _loaded = True
    env = os.environ.get("TDP_CONV_PLAN_DB", "")
    if env == "0":
        return
    load(C, env or DEFAULT_DB)
