#!/usr/bin/env python3
"""RCCL bus-bandwidth sweep over the native communicator (SURVEY.md §5.8 / §4.2 "comm" tier).

  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
      scripts/rccl_sweep.py [--min-kib 1] [--max-mib 256] [--iters 20]

One JSON line per (collective, size) on rank 0: all-reduce / reduce-scatter / all-gather bus
bandwidth (nccl-tests convention) from 1 KiB to 256 MiB in powers of 4, plus the bucket-plan
consequence for the toy MLP's two buckets (64.2 / 144 MiB). The same measurement runs in small
form inside bench.py at world size > 1 (diagnostics.busbw_GBps).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--min-kib", type=int, default=1)
    ap.add_argument("--max-mib", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    import tutorial_torch_distributed_data_parallel_amd as tdp
    from tutorial_torch_distributed_data_parallel_amd.parallel import commbench
    from tutorial_torch_distributed_data_parallel_amd.parallel import runtime as rt

    tdp.init_process_group("nccl")
    sizes, s = [], a.min_kib * 1024
    while s <= a.max_mib * 2 ** 20:
        sizes.append(s)
        s *= 4
    rows = commbench.collective_busbw(sizes, iters=a.iters, warmup=a.warmup)
    if rt.get_rank() == 0:
        for r in rows:
            print(json.dumps(r), flush=True)
    tdp.destroy_process_group()


if __name__ == "__main__":
    main()
