"""Input-gradient GEMM with B gathered from the channels_last weight (WTap) vs the dense
transposed-weight copy (the previous path: one ATen permute copy + dense B) on ResNet-50 /
AlexNet shapes. One JSON line per shape."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from tutorial_torch_distributed_data_parallel_amd._native import native


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / iters


C = native()
SHAPES = [  # (B, Cin, H, W, Cout, R, pad)
    (128, 256, 56, 56, 64, 1, 0), (128, 512, 28, 28, 128, 1, 0), (128, 1024, 14, 14, 256, 1, 0),
    (128, 2048, 7, 7, 512, 1, 0),
    (128, 64, 56, 56, 64, 3, 1), (128, 128, 28, 28, 128, 3, 1), (128, 256, 14, 14, 256, 3, 1),
    (128, 512, 7, 7, 512, 3, 1), (128, 64, 27, 27, 192, 5, 2), (128, 192, 13, 13, 384, 3, 1),
    (128, 384, 13, 13, 256, 3, 1), (128, 256, 13, 13, 256, 3, 1)]
for B, Cin, H, W, Cout, R, pd in SHAPES:
    w = (torch.randn(Cout, Cin, R, R, device="cuda") * 0.05).contiguous(
        memory_format=torch.channels_last)
    dy = torch.randn(B, Cout, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    xs = [B, Cin, H, W]
    dense = lambda: C.conv_nhwc_dgrad(dy, w.permute(2, 3, 0, 1).contiguous(), xs, R, R, 1, 1,
                                      pd, pd)
    wtap = lambda: C.conv_nhwc_dgrad_w(dy, w, xs, 1, 1, pd, pd)
    acc_out = torch.zeros(B, Cin, H, W, device="cuda").contiguous(
        memory_format=torch.channels_last)
    wacc = lambda: C.conv_nhwc_dgrad_w(dy, w, xs, 1, 1, pd, pd, out=acc_out, beta=1.0)
    torch.testing.assert_close(dense(), wtap(), atol=1e-3, rtol=1e-3)
    add = lambda: wtap().add_(acc_out)
    print(json.dumps({"shape": [B, Cin, H, W, Cout, R], "dense_copy_us": round(timeit(dense), 1),
                      "wtap_us": round(timeit(wtap), 1), "wtap_beta1_us": round(timeit(wacc), 1),
                      "wtap_then_add_us": round(timeit(add), 1)}), flush=True)
