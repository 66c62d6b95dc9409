"""RCCL bus-bandwidth measurements over the native communicator (SURVEY.md §5.8, §4.2 "comm" tier).

``collective_busbw`` times all-reduce / reduce-scatter / all-gather back to back on the current
stream and reports nccl-tests' bus bandwidth (algbw x 2(n-1)/n for all-reduce, x (n-1)/n for the
other two), which is what the 7 point-to-point xGMI links of a rank bound. ``ddp_comm_ms`` times
exactly the collectives one DDP step issues (the bucket plan of a model, sharded or not) with no
compute around them: the denominator of the overlap figure bench.py reports. Factored Linear
weights (DDP._factor_candidates) are timed as what they send: the factor all-gathers and the
all-gather of the updated parameters.
Used by ``scripts/rccl_sweep.py`` and, at world size > 1, by ``bench.py`` itself (the driver's
multi-GPU run is where the measurements come from).
"""
from __future__ import annotations

import torch

from . import runtime as rt


def _time(fn, iters: int, warmup: int) -> float:
    for _ in range(warmup):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def collective_busbw(sizes_bytes, ops=("all_reduce", "reduce_scatter", "all_gather"),
                     iters: int = 10, warmup: int = 3, dtype=torch.float32) -> list[dict]:
    comm = rt.comm()
    if comm is None:
        raise RuntimeError("collective_busbw needs the RCCL communicator")
    n, dev = comm.world, rt.device()
    esz = torch.tensor([], dtype=dtype).element_size()
    out = []
    for size in sizes_bytes:
        count = max(size // esz // n * n, n)
        buf = torch.ones(count, dtype=dtype, device=dev)
        part = buf[: count // n]
        for op in ops:
            if op == "all_reduce":
                ms = _time(lambda: comm.all_reduce(buf, "sum"), iters, warmup)
                factor = 2.0 * (n - 1) / n
            elif op == "reduce_scatter":
                ms = _time(lambda: comm.reduce_scatter(part, buf, "sum"), iters, warmup)
                factor = (n - 1) / n
            else:
                ms = _time(lambda: comm.all_gather(buf, part), iters, warmup)
                factor = (n - 1) / n
            nbytes = count * esz
            algbw = nbytes / (ms * 1e-3) / 1e9
            out.append({"op": op, "bytes": int(nbytes), "ms": round(ms, 4),
                        "algbw_GBps": round(algbw, 2), "busbw_GBps": round(algbw * factor, 2),
                        "n": n})
        del buf
    return out


def ddp_comm_ms(ddp, iters: int = 10, warmup: int = 3) -> float:
    """Milliseconds per step of the bucket collectives of ``ddp`` alone (its bucket bounds, its
    sharded or all-reduce schedule), on scratch buffers of the arena's size."""
    comm = rt.comm()
    if comm is None or not ddp._gpu:
        return 0.0
    W, r = ddp.world_size, ddp.rank
    g = torch.zeros_like(ddp.arena.grad)
    p = torch.zeros_like(ddp.arena.data)
    sharded = bool(ddp._fused_opt is not None and ddp._fused_shard)
    plan = []
    b = ddp._bounds
    # factored weights (DDP._factor_candidates): factor all-gathers + the parameter all-gather
    factored = {ddp._factor_bucket[i]: (ddp._factor_last_B[i],) + ddp._factor[i][:2]
                for i in ddp._factor if i in ddp._factor_last_B}
    quiet = {ddp._factor_bias_bucket[i] for i in ddp._factor
             if i in ddp._factor_last_B and i in ddp._factor_bias_bucket}
    fbufs = {k: (torch.zeros(W * B * o, device=g.device), torch.zeros(W * B * n, device=g.device))
             for k, (B, o, n) in factored.items()}
    for i in range(len(b) - 1):
        lo, hi = b[i], b[i + 1]
        if i in quiet:  # a factored bias: averaged from the gathered factors, no collective
            continue
        if i in factored:
            plan.append((lo, hi, -(i + 1)))
        elif sharded:
            s0, s1 = ddp._backend.owned_shard(lo, hi)
            cnt = s1 - s0
            plan.append((lo, hi, cnt))
        else:
            plan.append((lo, hi, 0))

    def step():
        for lo, hi, cnt in plan:
            if cnt < 0:  # factored bucket
                B, o, n = factored[-cnt - 1]
                ga, xa = fbufs[-cnt - 1]
                comm.all_gather(ga, ga[r * B * o: (r + 1) * B * o])
                comm.all_gather(xa, xa[r * B * n: (r + 1) * B * n])
                c = (hi - lo) // W
                comm.all_gather(p[lo: lo + W * c], p[lo + r * c: lo + (r + 1) * c])
            elif cnt > 0:
                comm.reduce_scatter(g[lo + r * cnt: lo + (r + 1) * cnt], g[lo: lo + W * cnt],
                                    "avg")
                if lo + W * cnt < hi:
                    comm.all_reduce(g[lo + W * cnt: hi], "avg")
                comm.all_gather(p[lo: lo + W * cnt], p[lo + r * cnt: lo + (r + 1) * cnt])
            else:
                comm.all_reduce(g[lo:hi], "avg")

    ms = _time(step, iters, warmup)
    del g, p, fbufs
    return ms
