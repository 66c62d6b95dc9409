"""Micro-benchmark of the classifier head + loss launches (toy MLP fc3: B = 128, 4096 -> 10).

    python scripts/bench_head.py [--iters 400]

Times, on one stream and replayed as hipGraphs of 20 launches each: the fused forward
(csrc/gemm_skinny.hip head_ce) with and without the training outputs (dlogits, dx + planes),
and the unfused launches it replaces (skinny head GEMM, ce_fwd with the unit-seed gradient,
head_bwd's input-gradient part). Prints one JSON line per variant (us per launch group)."""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=400)
    ap.add_argument("--B", type=int, default=128)
    ap.add_argument("--I", type=int, default=4096)
    a = ap.parse_args()
    import torch

    from tutorial_torch_distributed_data_parallel_amd._native import native
    from tutorial_torch_distributed_data_parallel_amd.ops.loss import _ticket

    C = native()
    B, I, O = a.B, a.I, 10
    x = torch.relu(torch.randn(B, I, device="cuda"))
    w = torch.randn(O, I, device="cuda") * 0.05
    b = torch.randn(O, device="cuda")
    y = torch.randint(0, O, (B,), device="cuda")
    acc = torch.zeros(3, device="cuda")
    lg = torch.empty(B, O, device="cuda")
    dx = torch.empty(B, I, device="cuda")
    dw = torch.empty(O, I, device="cuda")
    tk = _ticket(x.device)

    variants = {
        "head_ce train": lambda: C.head_ce(x, w, b, y, -100, 0.0, True, acc, with_grad=True,
                                           gate=x, planes=True, ticket=tk),
        "head_ce eval": lambda: C.head_ce(x, w, b, y, -100, 0.0, True, acc, with_grad=False,
                                          gate=None, planes=False, ticket=tk),
        "head_ce train, no planes": lambda: C.head_ce(x, w, b, y, -100, 0.0, True, acc,
                                                      with_grad=True, gate=x, planes=False,
                                                      ticket=tk),
        "skinny": lambda: C.gemm_f32(x, w, lg, True, True, bias=b),
        "ce_fwd": lambda: C.ce_fwd(lg, y, -100, 0.0, True, acc, with_grad=True),
    }
    d = C.ce_fwd(lg, y, -100, 0.0, True, acc, with_grad=True)[2]
    variants["head_bwd dx+dw"] = lambda: C.head_bwd(d, x, w, dx, dw, gate=x, planes=True)
    variants["head_bwd dw only"] = lambda: C.head_bwd(d, x, w, None, dw)
    variants["skinny+ce_fwd+head_bwd"] = lambda: (variants["skinny"](), variants["ce_fwd"](),
                                                  variants["head_bwd dx+dw"]())
    variants["head_ce+head_bwd dw"] = lambda: (variants["head_ce train"](),
                                               variants["head_bwd dw only"]())
    s = torch.cuda.Stream()
    for name, fn in variants.items():
        with torch.cuda.stream(s):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(20):
                    fn()
            for _ in range(5):
                g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(a.iters // 20):
                g.replay()
            e1.record(s)
            torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000.0 / (a.iters // 20 * 20)
        print(json.dumps({"variant": name, "us": round(us, 2), "B": B, "I": I}), flush=True)


if __name__ == "__main__":
    main()
