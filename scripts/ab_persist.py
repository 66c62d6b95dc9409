"""A/B of the persistent plain GEMM (resident grid, next tile's operands prefetched under the
epilogue) vs one workgroup per tile, on ResNet-50 / AlexNet conv shapes and plain GEMMs,
interleaved in one process (min of 5). Also checks both give identical results."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from tutorial_torch_distributed_data_parallel_amd import ops
from tutorial_torch_distributed_data_parallel_amd._native import native

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ab_cvec import timeit  # noqa: E402

C = native()
B = 128
SHAPES = [(64, 56, 64, 3, 1), (128, 28, 128, 3, 1), (256, 14, 256, 3, 1), (512, 7, 512, 3, 1),
          (64, 56, 256, 1, 1), (256, 56, 64, 1, 1), (128, 28, 512, 1, 1), (512, 28, 128, 1, 1),
          (1024, 14, 256, 1, 1), (256, 14, 1024, 1, 1), (256, 56, 128, 1, 1),
          (64, 27, 192, 5, 1), (192, 13, 384, 3, 1), (384, 13, 256, 3, 1)]
for Cin, H, Cout, R, st in SHAPES:
    pd = R // 2
    x = torch.randn(B, Cin, H, H, device="cuda").contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, R, R, device="cuda") * 0.05).contiguous(
        memory_format=torch.channels_last)
    dy = torch.randn(B, Cout, H, H, device="cuda").contiguous(memory_format=torch.channels_last)
    fwd = lambda: ops.conv2d(x, w, None, st, pd)
    dgr = lambda: C.conv_nhwc_dgrad_w(dy, w, [B, Cin, H, H], 1, 1, pd, pd)
    for tag, fn in (("fwd", fwd), ("dgrad", dgr)):
        C.gemm_f32_set_persist(False)
        ref = fn().clone()
        C.gemm_f32_set_persist(True)
        got = fn()
        diff = (got - ref).abs().max().item()
        res = {0: [], 1: []}
        for _ in range(5):
            for m in (0, 1):
                C.gemm_f32_set_persist(bool(m))
                res[m].append(timeit(fn))
        C.gemm_f32_set_persist(False)
        print(json.dumps({"shape": [Cin, H, Cout, R], "pass": tag, "tiles_us": round(min(res[0]), 1),
                          "persist_us": round(min(res[1]), 1), "max_abs_diff": diff}), flush=True)
for (M, N, K) in [(401408, 256, 64), (100352, 512, 128), (8192, 8192, 512), (128 * 1024, 1024, 256)]:
    A = torch.randn(M, K, device="cuda")
    Bm = torch.randn(N, K, device="cuda")
    out = torch.empty(M, N, device="cuda")
    fn = lambda: C.gemm_f32(A, Bm, out, True, True)
    res = {0: [], 1: []}
    for _ in range(5):
        for m in (0, 1):
            C.gemm_f32_set_persist(bool(m))
            res[m].append(timeit(fn))
    C.gemm_f32_set_persist(False)
    print(json.dumps({"gemm": [M, N, K], "tiles_us": round(min(res[0]), 1),
                      "persist_us": round(min(res[1]), 1)}), flush=True)
