"""rocprofv3 --kernel-trace CSV -> how much collective (RCCL) kernel time ran concurrently with
compute kernels.

python scripts/overlap_report.py <kernel_trace.csv> [--last-steps N --step-marker SUBSTR] > out.md

A kernel is a collective when its name contains "nccl"/"rccl" (RCCL's device kernels are
``ncclDevKernel_*``). For every collective kernel the report gives the share of its [start, end)
interval covered by the union of the compute kernels' intervals; the total is the duration-weighted
share over all collective kernels. Without a step marker the whole trace is used; with one, only
the window from the N-th-last occurrence of the marker kernel (the first kernel of a step, e.g.
``gather_batch``) to the end of the trace.
"""
from __future__ import annotations

import argparse
import csv
import re
import sys


def _col(row, *names):
    for n in names:
        if n in row:
            return row[n]
    raise KeyError(f"none of {names} in {list(row)}")


def load(path):
    out = []
    for r in csv.DictReader(open(path)):
        name = _col(r, "Kernel_Name", "KernelName", "Name")
        t0 = int(_col(r, "Start_Timestamp", "BeginNs", "Start"))
        t1 = int(_col(r, "End_Timestamp", "EndNs", "End"))
        q = r.get("Queue_Id") or r.get("Stream_Id") or ""
        out.append((t0, t1, name, q))
    out.sort()
    return out


def is_coll(name: str) -> bool:
    n = name.lower()
    return "nccl" in n or "rccl" in n or "onerankreduce" in n


def short(name: str, n: int = 60) -> str:
    name = re.sub(r"^void ", "", name).replace("(anonymous namespace)::", "")
    return name.split("(")[0][:n]


def union(intervals):
    iv = sorted(intervals)
    merged = []
    for a, b in iv:
        if merged and a <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], b)
        else:
            merged.append([a, b])
    return merged


def covered(a, b, merged):
    tot = 0
    for x, y in merged:
        if y <= a:
            continue
        if x >= b:
            break
        tot += min(b, y) - max(a, x)
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step-marker", default=None)
    ap.add_argument("--last-steps", type=int, default=0)
    ap.add_argument("--title", default="collective / compute overlap")
    ap.add_argument("--by-queue", action="store_true",
                    help="side-stream work = EVERY kernel on the hardware queue(s) that run the "
                         "collectives (the factored jobs' GEMMs and updates too), compute = the "
                         "kernels of every other queue")
    a = ap.parse_args()
    ks = load(a.trace)
    # the hardware queue(s) that run collectives anywhere in the trace (a short window may hold
    # none of the few collective KERNELS: a one-rank all-gather is a copy on that queue)
    side_q = {k[3] for k in ks if is_coll(k[2])}
    if len(side_q) > 1:  # a collective issued on the compute stream (eager): not a side queue
        busy = {}
        for k in ks:
            busy[k[3]] = busy.get(k[3], 0) + k[1] - k[0]
        side_q.discard(max(side_q, key=lambda q: busy.get(q, 0)))
    if a.step_marker and a.last_steps:
        starts = [k[0] for k in ks if a.step_marker in k[2]]
        if len(starts) >= a.last_steps:
            t_lo = starts[-a.last_steps]
            ks = [k for k in ks if k[0] >= t_lo]
    if a.by_queue:
        side = lambda k: k[3] in side_q  # noqa: E731
    else:
        side = lambda k: is_coll(k[2])  # noqa: E731
    coll = [k for k in ks if side(k)]
    comp = union([(k[0], k[1]) for k in ks if not side(k)])
    span = (ks[-1][1] - ks[0][0]) if ks else 0
    print(f"# {a.title}\n")
    print(f"Source: `{a.trace}`; window {span / 1e6:.3f} ms, {len(ks)} kernels, "
          f"{len(coll)} collective kernels"
          + (f" (last {a.last_steps} steps from `{a.step_marker}`)" if a.step_marker else "")
          + ".\n")
    if not coll:
        print("No collective kernels in the window.")
        return
    tot = sum(k[1] - k[0] for k in coll)
    hid = sum(covered(k[0], k[1], comp) for k in coll)
    busy = sum(y - x for x, y in comp)
    print(f"Collective kernel time {tot / 1e3:.1f} us, of which {hid / 1e3:.1f} us "
          f"({100.0 * hid / max(tot, 1):.1f} %) ran while a compute kernel was executing; "
          f"compute busy {busy / 1e6:.3f} ms of the window.\n")
    print("| collective kernel | start (us, rel.) | dur us | overlapped % | concurrent compute kernels |")
    print("|---|---|---|---|---|")
    base = ks[0][0]
    for k in coll[:60]:
        d = k[1] - k[0]
        c = covered(k[0], k[1], comp)
        names = sorted({short(x[2], 40) for x in ks
                        if not side(x) and x[0] < k[1] and x[1] > k[0]})
        print(f"| `{short(k[2])}` | {(k[0] - base) / 1e3:.1f} | {d / 1e3:.1f} | "
              f"{100.0 * c / max(d, 1):.1f} | {', '.join('`%s`' % n for n in names[:4])} |")


if __name__ == "__main__":
    sys.exit(main())
