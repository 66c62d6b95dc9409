"""Does a captured fork/join step keep its side-stream branch concurrent on replay?

The pattern of the reducer inside a captured DDP step: a compute chain on the capture stream,
and after segment k a fork to the communicator's stream (wait on an event recorded after segment
k, then the bucket's collective + update), joined back at the end. Each node here is a
``torch.cuda._sleep`` spin (one thread: concurrency shows up as wall time, not as shared CUs).

  order "comm_first":    record ev; side.wait(ev); side: sleep; then main: next segment
  order "compute_first": record ev; main: next segment; then side.wait(ev); side: sleep
  order "marker":        record ev; main: tiny node; side.wait(ev); side: sleep; main: segment

Fully concurrent replay takes ~ (forks + 1) * T; a side branch that lands on the compute
chain's hardware queue serialises with it (up to 2x). Prints one JSON line per order.
"""
from __future__ import annotations

import json
import sys
import time

import torch


def build(order: str, forks: int, cycles: int):
    main = torch.cuda.Stream()
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.stream(main):
        with torch.cuda.graph(g, stream=main):
            side.wait_stream(main)
            torch.cuda._sleep(cycles)
            for _ in range(forks):
                ev = torch.cuda.Event()
                ev.record(main)
                if order == "marker":
                    torch.cuda._sleep(1)  # tiny node: the compute chain's first edge
                    side.wait_event(ev)
                    with torch.cuda.stream(side):
                        torch.cuda._sleep(cycles)
                    torch.cuda._sleep(cycles)
                elif order == "comm_first":
                    side.wait_event(ev)
                    with torch.cuda.stream(side):
                        torch.cuda._sleep(cycles)
                    torch.cuda._sleep(cycles)
                else:
                    torch.cuda._sleep(cycles)
                    side.wait_event(ev)
                    with torch.cuda.stream(side):
                        torch.cuda._sleep(cycles)
            main.wait_stream(side)
    return g


def timed(g, iters=5):
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1000.0 / iters


def main():
    forks = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    cycles = 2_000_000
    # one spin alone
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    torch.cuda._sleep(cycles)
    e.record()
    torch.cuda.synchronize()
    s.record()
    torch.cuda._sleep(cycles)
    e.record()
    torch.cuda.synchronize()
    t_one = s.elapsed_time(e)
    for order in ("comm_first", "compute_first", "marker"):
        g = build(order, forks, cycles)
        ms = timed(g)
        print(json.dumps({"order": order, "forks": forks, "spin_ms": round(t_one, 3),
                          "replay_ms": round(ms, 3),
                          "concurrent_ms": round((forks + 1) * t_one, 3),
                          "serial_ms": round((2 * forks + 1) * t_one, 3)}), flush=True)


if __name__ == "__main__":
    main()
