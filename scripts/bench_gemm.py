"""GEMM microbenchmark: native fp32 kernels (fast / generic) vs torch.mm (hipBLASLt) on the
toy-MLP shapes. Interleaved rounds in one process (guide §5.4 rule 24); random operands."""
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from tutorial_torch_distributed_data_parallel_amd._native import native  # noqa: E402

C = native()
dev = "cuda"
# (name, M, N, K, a_kcontig, b_kcontig)
SHAPES = [("fc1_fwd", 128, 4096, 9216, True, True), ("fc2_fwd", 128, 4096, 4096, True, True),
          ("fc3_fwd", 128, 10, 4096, True, True), ("fc2_dgrad", 128, 4096, 4096, True, False),
          ("fc1_wgrad", 4096, 9216, 128, False, False), ("fc2_wgrad", 4096, 4096, 128, False, False),
          ("sq4096", 4096, 4096, 4096, True, True)]


def mk(M, N, K, ak, bk):
    A = torch.randn((M, K) if ak else (K, M), device=dev)
    B = torch.randn((N, K) if bk else (K, N), device=dev)
    return A, B, torch.empty(M, N, device=dev)


def torch_mm(A, B, out, ak, bk):
    a = A if ak else A.t()
    b = B.t() if bk else B
    torch.mm(a, b, out=out)


def timeit(fn, reps=20):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps * 1000.0  # us


SWEEP = {  # (fn, splits, stages) variants of the fast kernel to compare per shape
    "fc1_fwd": [(1, 4, 3), (1, 8, 3), (1, 8, 2), (2, 8, 2), (2, 16, 2), (1, 16, 3)],
    "fc2_fwd": [(1, 4, 3), (1, 8, 3), (2, 8, 2), (1, 16, 2)],
    "fc2_dgrad": [(1, 4, 3), (1, 8, 3), (2, 8, 2), (2, 16, 2)],
    "fc1_wgrad": [(2, 1, 2), (2, 1, 3), (1, 1, 2)],
    "fc2_wgrad": [(2, 1, 2), (1, 1, 2)],
}

res = {}
for name, M, N, K, ak, bk in SHAPES:
    A, B, out = mk(M, N, K, ak, bk)
    fl = 2.0 * M * N * K
    row = {"plan": C.gemm_f32_plan(M, N, K, False, C.num_cus(0))}
    for rnd in range(3):
        for impl in ("fast", "generic", "torch"):
            if impl == "torch":
                f = lambda: torch_mm(A, B, out, ak, bk)
            else:
                mode = 0 if impl == "fast" else 1
                def f(mode=mode):
                    C.gemm_f32_set_mode(mode)
                    C.gemm_f32(A, B, out, ak, bk)
                    C.gemm_f32_set_mode(0)
            us = timeit(f)
            row.setdefault(impl, []).append(us)
    for v in SWEEP.get(name, []):
        A2, B2, out2 = A, B, out
        C.gemm_f32_set_override(*v)
        try:
            us = min(timeit(lambda: C.gemm_f32(A2, B2, out2, ak, bk)) for _ in range(3))
        finally:
            C.gemm_f32_set_override(0, 0, 0)
        row[f"fn{v[0]}_s{v[1]}_st{v[2]}_us"] = round(us, 1)
    for impl in ("fast", "generic", "torch"):
        us = min(row[impl])
        row[impl + "_us"] = round(us, 1)
        row[impl + "_tflops"] = round(fl / us / 1e6, 1)
        del row[impl]
    res[name] = row
    print(name, json.dumps(row), flush=True)
