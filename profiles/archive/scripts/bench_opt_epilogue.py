#!/usr/bin/env python3
"""Micro-benchmark of the weight-gradient GEMM with the optimizer epilogue (world size 1).

For the toy MLP's fc1 / fc2 weight-gradient shapes it times, per tile width / pipeline depth:
  * the plain wgrad GEMM (stores dW) followed by the flat SGD kernel over the same range, and
  * the wgrad GEMM whose epilogue applies SGD (dW never stored),
and reports the HBM roofline of each (bytes / 6 TB/s) next to the fp32 MFMA time.

  python scripts/bench_opt_epilogue.py
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import tutorial_torch_distributed_data_parallel_amd as tdp  # noqa: E402
from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP  # noqa: E402


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / iters


def main():
    tdp.init_process_group("nccl", rank=0, world_size=1, local_rank=0)
    C = tdp._native.native()
    dev = torch.device("cuda", 0)
    model = ToyMLP(device=dev)
    ddp = tdp.DDP(model, device_ids=[0])
    opt = tdp.optim.SGD(ddp.parameters(), lr=0.01, momentum=0.9)
    assert ddp.register_fused_optimizer(opt) and ddp._epi_on
    x = torch.randn(128, 9216, device=dev)
    y = torch.randint(0, 10, (128,), device=dev)
    for _ in range(2):  # creates the momentum buffers, leaves the first-step flag cleared
        tdp.ops.cross_entropy(ddp(x), y).backward()
    torch.cuda.synchronize()
    be = ddp._backend
    mom = opt._flat_bufs[id(ddp.arena)]["momentum_buffer"]
    out = []
    for name, (M, N) in {"fc1": (4096, 9216), "fc2": (4096, 4096)}.items():
        w = getattr(model, name).weight
        i = ddp.arena.index(w)
        off = ddp.arena.offsets[i]
        g = torch.randn(128, M, device=dev)   # dY, stored [K=batch][M]
        a = torch.randn(128, N, device=dev)   # X,  stored [K][N]
        dw = ddp.arena.grad[off: off + M * N].view(M, N)
        p = ddp.arena.data[off: off + M * N]
        b = mom[off: off + M * N]
        flops = 2.0 * M * N * 128
        for fn, st, wgs in ((0, 0, 2), (1, 2, 2), (1, 2, 3), (1, 3, 2), (2, 2, 2)):
            C.gemm_f32_set_override(fn, 0, st)
            C.gemm_f32_set_opt_variant(wgs=wgs)  # persistent epilogue grid: workgroups per CU
            t_gemm = timed(lambda: C.gemm_f32(g, a, dw, False, False))
            t_sgd = timed(lambda: C.sgd_flat(p, dw.view(-1), b, 1e-6, 0.9, 0.0, 0.0, False, False,
                                             False, 1.0))
            t_epi = timed(lambda: C.gemm_f32_opt(g, a, dw, False, False, be, off))
            rec = {"layer": name, "fn": fn, "stages": st, "wgs": wgs, "gemm_us": round(t_gemm, 1),
                   "sgd_us": round(t_sgd, 1), "gemm+sgd_us": round(t_gemm + t_sgd, 1),
                   "epilogue_us": round(t_epi, 1),
                   "mfma_floor_us": round(flops / 157e12 * 1e6, 1),
                   "hbm_floor_epi_us": round(4 * 4 * M * N / 6e12 * 1e6, 1)}
            out.append(rec)
            print(json.dumps(rec), flush=True)
    C.gemm_f32_set_override(0, 0, 0)
    C.gemm_f32_set_opt_variant(wgs=2)
    tdp.destroy_process_group()


if __name__ == "__main__":
    main()
