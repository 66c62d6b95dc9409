"""PMC probe: 4096^3 split-bf16 GEMM, the 256x256 kernel (gemm_emu8) then the 128x128 fast
kernel, 10 launches each (rocprofv3 --pmc attributes counters per dispatch)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/dev/", 1)[0])
from tutorial_torch_distributed_data_parallel_amd._native import native  # noqa: E402

C = native()
A = torch.randn(4096, 4096, device="cuda")
B = torch.randn(4096, 4096, device="cuda")
out = torch.empty(4096, 4096, device="cuda")
for _ in range(10):
    C.gemm_emu8(A, B, out, True)
C.gemm_f32_set_mode(2)
for _ in range(10):
    C.gemm_f32(A, B, out, True, True)
torch.cuda.synchronize()
