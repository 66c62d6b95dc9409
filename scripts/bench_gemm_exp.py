"""Timing experiment (numerically wrong by design): how fast would the split-bf16 fp32 GEMM run
if the A (bit 0) and/or B (bit 1) fragments came pre-split, i.e. without their VALU split?
Bounds the gain of pre-split operand planes. One JSON line per shape: microseconds per mode.

python scripts/bench_gemm_exp.py"""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from tutorial_torch_distributed_data_parallel_amd._native import native  # noqa: E402

C = native()
SHAPES = [("fc1_fwd", 128, 4096, 9216, True, True), ("fc2_fwd", 128, 4096, 4096, True, True),
          ("fc2_dgrad", 128, 4096, 4096, True, False), ("sq4096", 4096, 4096, 4096, True, True),
          ("r50_1x1b", 25088, 1024, 256, True, True), ("conv_like", 21632, 384, 1728, True, True)]


def timeit(fn, reps=20):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps * 1000.0


x = torch.randn(4096, 4096, device="cuda")
for _ in range(40):
    torch.mm(x, x)
torch.cuda.synchronize()
for name, M, N, K, ak, bk in SHAPES:
    A = torch.randn((M, K) if ak else (K, M), device="cuda")
    B = torch.randn((N, K) if bk else (K, N), device="cuda")
    out = torch.empty(M, N, device="cuda")
    fl = 2.0 * M * N * K
    best = {}
    for rnd in range(3):
        for bits in (0, 1, 2, 3):
            C.gemm_f32_set_exp(bits)
            us = timeit(lambda: C.gemm_f32(A, B, out, ak, bk), reps=10 if fl > 1e12 else 30)
            best[bits] = min(best.get(bits, 1e30), us)
    C.gemm_f32_set_exp(0)
    row = {f"exp{b}_us": round(v, 1) for b, v in best.items()}
    row.update({f"exp{b}_tflops": round(fl / v / 1e6, 1) for b, v in best.items()})
    row["plan"] = C.gemm_f32_plan(M, N, K, False, C.num_cus(0))
    print(json.dumps({name: row}), flush=True)
