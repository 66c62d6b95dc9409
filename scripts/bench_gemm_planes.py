"""Planes-A skinny GEMM (csrc/gemm_planes.hip) vs the split-bf16 fast GEMM on the toy-MLP's
forward / input-gradient shapes: the GEMM alone (planes made beforehand), the split_planes pass
alone, and the fast kernel's whole call (its split-K reduce included in both). Interleaved rounds
in one process, best of 3; prints one JSON line per shape."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from tutorial_torch_distributed_data_parallel_amd._native import native  # noqa: E402

C = native()
dev = "cuda"
# (name, M, N, K, b_kcontig)
SHAPES = [("fc1_fwd", 128, 4096, 9216, True), ("fc2_fwd", 128, 4096, 4096, True),
          ("fc2_dgrad", 128, 4096, 4096, False), ("b256_fc1_fwd", 256, 4096, 9216, True)]


def timeit(fn, reps=30):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps * 1000.0  # us


for name, M, N, K, bk in SHAPES:
    A = torch.randn(M, K, device=dev)
    B = torch.randn((N, K) if bk else (K, N), device=dev)
    out = torch.empty(M, N, device=dev)
    P = C.split_planes(A)
    fl = 2.0 * M * N * K
    row = {"plan": C.gemm_planes_plan(M, N, K, C.num_cus(0))}
    t = {"planes": [], "split": [], "fast": []}
    for _ in range(3):
        t["planes"].append(timeit(lambda: C.gemm_planes(P, B, out, bk)))
        t["split"].append(timeit(lambda: C.split_planes(A)))
        t["fast"].append(timeit(lambda: C.gemm_f32(A, B, out, True, bk)))
    for k, v in t.items():
        row[k + "_us"] = round(min(v), 1)
    row["planes_tflops"] = round(fl / row["planes_us"] / 1e6, 1)
    row["fast_tflops"] = round(fl / row["fast_us"] / 1e6, 1)
    print(name, json.dumps(row), flush=True)
