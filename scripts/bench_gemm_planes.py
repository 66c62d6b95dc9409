"""Pre-split planes GEMM (csrc/gemm_planes.hip, split pass included) vs the in-kernel split
fast GEMM on compute-bound shapes: square GEMMs and the factored weight gradient of W ranks
(dW[out][in] = g_all^T x_all, depth W*B, both operands stored [K][.]). One JSON line per shape.

python scripts/bench_gemm_planes.py"""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from tutorial_torch_distributed_data_parallel_amd._native import native  # noqa: E402

C = native()
SHAPES = [("sq4096", 4096, 4096, 4096, True, True), ("sq8192", 8192, 8192, 8192, True, True),
          ("sq4096_nn", 4096, 4096, 4096, False, False),
          ("factor_w4_fc1", 4096, 9216, 512, False, False),
          ("factor_w8_fc1", 4096, 9216, 1024, False, False),
          ("factor_w4_fc2", 4096, 4096, 512, False, False)]


def timeit(fn, reps=10):
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
        best["fast_split"] = min(best.get("fast_split", 1e30),
                                 timeit(lambda: C.gemm_f32(A, B, out, ak, bk)))
        best["planes_total"] = min(best.get("planes_total", 1e30),
                                   timeit(lambda: C.gemm_f32_planes(A, B, out, ak, bk)))
        best["split_only"] = min(best.get("split_only", 1e30),
                                 timeit(lambda: (C.split_planes(A, ak), C.split_planes(B, bk))))
    row = {k + "_us": round(v, 1) for k, v in best.items()}
    row.update({k + "_tflops": round(fl / v / 1e6, 1) for k, v in best.items() if k != "split_only"})
    row["planes_gemm_only_tflops"] = round(fl / (best["planes_total"] - best["split_only"]) / 1e6, 1)
    print(json.dumps({name: row}), flush=True)
