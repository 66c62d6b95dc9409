"""Fast-GEMM products A/B: split-bf16 emulation (6 bf16 MFMAs per 32x32x16 step) vs the native
v_mfma_f32_32x32x2_f32 path, on the toy-MLP shapes and a square reference shape, interleaved in
one process. One JSON line per shape: microseconds and TFLOP/s of each, and the plan.

python scripts/bench_gemm_emu.py"""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from tutorial_torch_distributed_data_parallel_amd._native import native  # noqa: E402

C = native()
dev = "cuda"
SHAPES = [("fc1_fwd", 128, 4096, 9216, True, True), ("fc2_fwd", 128, 4096, 4096, True, True),
          ("fc2_dgrad", 128, 4096, 4096, True, False),
          ("fc1_wgrad", 4096, 9216, 128, False, False), ("fc2_wgrad", 4096, 4096, 128, False, False),
          ("sq4096", 4096, 4096, 4096, True, True), ("sq8192_nt", 8192, 8192, 8192, True, False),
          ("r50_1x1", 100352, 256, 64, True, True), ("r50_1x1b", 25088, 1024, 256, True, True)]


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


# device clock warm-up (power-management ramp)
x = torch.randn(4096, 4096, device=dev)
for _ in range(40):
    torch.mm(x, x)
torch.cuda.synchronize()

for name, M, N, K, ak, bk in SHAPES:
    A = torch.randn((M, K) if ak else (K, M), device=dev)
    B = torch.randn((N, K) if bk else (K, N), device=dev)
    out = torch.empty(M, N, device=dev)
    fl = 2.0 * M * N * K
    row = {"shape": [M, N, K, ak, bk], "plan": C.gemm_f32_plan(M, N, K, False, C.num_cus(0))}
    best = {}
    for rnd in range(3):
        for emu in (True, False):
            C.gemm_f32_set_emu(emu)
            us = timeit(lambda: C.gemm_f32(A, B, out, ak, bk), reps=10 if fl > 1e12 else 20)
            key = "emu" if emu else "f32"
            best[key] = min(best.get(key, 1e30), us)
    C.gemm_f32_set_emu(True)
    for k, us in best.items():
        row[k + "_us"] = round(us, 1)
        row[k + "_tflops"] = round(fl / us / 1e6, 1)
    row["speedup"] = round(best["f32"] / best["emu"], 2)
    print(json.dumps({name: row}), flush=True)
