"""Split-K / tile sweep of the tensor-sharded step's GEMM shapes at W = 8 (fast kernel overrides,
gemm_f32_set_override): which plan the heuristic picks and what each plan measures.

python scripts/bench_tp_gemms.py"""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from tutorial_torch_distributed_data_parallel_amd._native import native  # noqa: E402

C = native()
dev = "cuda"
# name, M, N, K, A K-contiguous, B K-contiguous
SHAPES = [("dW1", 512, 9216, 1024, False, False), ("dW2", 4096, 512, 1024, False, False),
          ("dH1", 1024, 512, 4096, True, False), ("dW1_kk", 512, 9216, 1024, True, True)]


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


x = torch.randn(4096, 4096, device=dev)
for _ in range(40):
    x @ x
for name, M, N, K, ak, bk in SHAPES:
    A = torch.randn((M, K) if ak else (K, M), device=dev)
    B = torch.randn((N, K) if bk else (K, N), device=dev)
    out = torch.empty(M, N, device=dev)
    res = {}
    for fn in (1, 2):
        for sp in (1, 2, 3, 4, 6, 8):
            C.gemm_f32_set_override(fn, sp, 0)
            try:
                res[f"fn{fn}_s{sp}"] = round(min(timeit(lambda: C.gemm_f32(A, B, out, ak, bk))
                                                 for _ in range(2)), 1)
            except RuntimeError as e:
                res[f"fn{fn}_s{sp}"] = str(e)[:40]
    C.gemm_f32_set_override(0, 0, 0)
    res["auto"] = round(min(timeit(lambda: C.gemm_f32(A, B, out, ak, bk)) for _ in range(2)), 1)
    best = min((v, k) for k, v in res.items() if isinstance(v, float))
    print(json.dumps({name: {"shape": [M, N, K, ak, bk], "best": best[1],
                             "best_tflops": round(2 * M * N * K / best[0] / 1e6, 1), **res}}),
          flush=True)
