"""A/B of the fast GEMM's block rows (128 vs 256 = FM 4) on conv forward / input-gradient shapes,
toggled in one process and interleaved (min of 5): one JSON line per (shape, pass). Also checks the
two agree numerically."""
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
B = int(os.environ.get("AB_BATCH", "128"))
SHAPES = [(64, 56, 64, 3, 1), (128, 28, 128, 3, 1), (256, 14, 256, 3, 1), (512, 7, 512, 3, 1),
          (64, 56, 256, 1, 1), (256, 56, 64, 1, 1), (128, 28, 512, 1, 1), (1024, 14, 256, 1, 1),
          (256, 56, 128, 1, 1), (64, 27, 192, 5, 1), (192, 13, 384, 3, 1)]
for Cin, H, Cout, R, st in SHAPES:
    pd = R // 2
    x = torch.randn(B, Cin, H, H, device="cuda").contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, R, R, device="cuda") * 0.05).contiguous(
        memory_format=torch.channels_last)
    P = (H + 2 * pd - R) // st + 1
    dy = torch.randn(B, Cout, P, P, device="cuda").contiguous(memory_format=torch.channels_last)
    fwd = lambda: ops.conv2d(x, w, None, st, pd)
    dgr = lambda: C.conv_nhwc_dgrad_w(dy, w, [B, Cin, H, H], 1, 1, pd, pd)
    for tag, fn in (("fwd", fwd), ("dgrad", dgr)):
        C.gemm_f32_set_bm(128)
        ref = fn().clone()
        C.gemm_f32_set_bm(256)
        got = fn()
        err = (got - ref).abs().max().item()
        res = {128: [], 256: []}
        for _ in range(5):
            for bm in (128, 256):
                C.gemm_f32_set_bm(bm)
                res[bm].append(timeit(fn))
        C.gemm_f32_set_bm(0)
        print(json.dumps({"shape": [Cin, H, Cout, R], "pass": tag, "bm128_us": round(min(res[128]), 1),
                          "bm256_us": round(min(res[256]), 1), "max_abs_diff": err}), flush=True)
