"""Toy-MLP GEMM plan sweep: forward fc1 / fc2 and the fc2 input gradient at the headline shapes,
over (FN, split-K, stages) overrides vs the planner (min of 5 x 20 launches)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from tutorial_torch_distributed_data_parallel_amd._native import native

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ab_cvec import timeit  # noqa: E402

C = native()
B = 128
CASES = [("fc1_fwd", B, 4096, 9216, True, True), ("fc2_fwd", B, 4096, 4096, True, True),
         ("fc2_dgrad", B, 4096, 4096, True, False)]
for tag, M, N, K, ak, bk in CASES:
    A = torch.randn(M, K, device="cuda")
    Bm = torch.randn(N, K, device="cuda") if bk else torch.randn(K, N, device="cuda")
    out = torch.empty(M, N, device="cuda")
    fn = lambda: C.gemm_f32(A, Bm, out, ak, bk)
    cands = [(0, 0, 0)] + [(f, s, st) for f in (1, 2) for s in (2, 4, 6, 8, 12, 16, 24, 32)
                            for st in (2, 3)]
    res = {}
    for _ in range(4):
        for c in cands:
            C.gemm_f32_set_override(*c)
            res.setdefault(c, []).append(timeit(fn))
    C.gemm_f32_set_override(0, 0, 0)
    t = {k: min(v) for k, v in res.items()}
    best = sorted(t, key=t.get)[:5]
    print(json.dumps({"gemm": tag, "auto_us": round(t[(0, 0, 0)], 1),
                      "plan": C.gemm_f32_plan(M, N, K, False, 256),
                      "best": [[list(b), round(t[b], 1)] for b in best]}), flush=True)
