"""Probe for rocprofv3: three launches of the planes GEMM on the toy-MLP fc1 forward and fc2
input-gradient shapes (planes made beforehand), then three of the fast split-bf16 GEMM."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from tutorial_torch_distributed_data_parallel_amd._native import native  # noqa: E402

C = native()
for M, N, K, bk in [(128, 4096, 9216, True), (128, 4096, 4096, False)]:
    A = torch.randn(M, K, device="cuda")
    B = torch.randn((N, K) if bk else (K, N), device="cuda")
    out = torch.empty(M, N, device="cuda")
    P = C.split_planes(A)
    for _ in range(3):
        C.gemm_planes(P, B, out, bk)
    torch.cuda.synchronize()
    for _ in range(3):
        C.gemm_f32(A, B, out, True, bk)
    torch.cuda.synchronize()
