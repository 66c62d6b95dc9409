"""A/B of the fast GEMM tile width on N = 128 convolution GEMMs: the planner's 64-wide tile (FN 1)
vs the 128-wide tile (FN 2), interleaved in one process (min of 5)."""
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
SHAPES = [(128, 28, 128, 3, 1), (256, 56, 128, 1, 1), (128, 28, 512, 1, 1), (512, 28, 128, 1, 1),
          (64, 56, 64, 3, 1), (64, 56, 256, 1, 1)]
for Cin, H, Cout, R, st in SHAPES:
    pd = R // 2
    x = torch.randn(B, Cin, H, H, device="cuda").contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, R, R, device="cuda") * 0.05).contiguous(
        memory_format=torch.channels_last)
    dy = torch.randn(B, Cout, H, H, device="cuda").contiguous(memory_format=torch.channels_last)
    fwd = lambda: ops.conv2d(x, w, None, st, pd)
    dgr = lambda: C.conv_nhwc_dgrad_w(dy, w, [B, Cin, H, H], 1, 1, pd, pd)
    for tag, fn in (("fwd", fwd), ("dgrad", dgr)):
        res = {}
        for _ in range(5):
            for mode in ("auto", "fn2", "fn1s3"):
                C.gemm_f32_set_override(*{"auto": (0, 0, 0), "fn2": (2, 0, 0),
                                          "fn1s3": (1, 0, 3)}[mode])
                res.setdefault(mode, []).append(timeit(fn))
        C.gemm_f32_set_override(0, 0, 0)
        print(json.dumps({"shape": [Cin, H, Cout, R], "pass": tag,
                          **{k + "_us": round(min(v), 1) for k, v in res.items()}}), flush=True)
