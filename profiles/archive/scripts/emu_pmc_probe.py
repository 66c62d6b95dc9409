"""PMC probe: a few fast-GEMM launches with split-bf16 products, then native f32 (same shapes)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from tutorial_torch_distributed_data_parallel_amd._native import native  # noqa: E402

C = native()
for M, N, K, ak, bk in [(4096, 4096, 4096, True, True), (4096, 9216, 128, False, False)]:
    A = torch.randn((M, K) if ak else (K, M), device="cuda")
    B = torch.randn((N, K) if bk else (K, N), device="cuda")
    out = torch.empty(M, N, device="cuda")
    for emu in (True, False):
        C.gemm_f32_set_emu(emu)
        for _ in range(3):
            C.gemm_f32(A, B, out, ak, bk)
        torch.cuda.synchronize()
C.gemm_f32_set_emu(True)
