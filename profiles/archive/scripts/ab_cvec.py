"""A/B of the GEMM's row-vector (LDS-staged) output stores on ResNet-50 conv shapes, toggled in
one process and interleaved (min of 5 alternations): one JSON line per (shape, pass)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from tutorial_torch_distributed_data_parallel_amd import ops
from tutorial_torch_distributed_data_parallel_amd._native import native


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / iters


def main():
    C = native()
    B = 128
    SHAPES = [(64, 56, 64, 3, 1), (128, 28, 128, 3, 1), (256, 14, 256, 3, 1), (512, 7, 512, 3, 1),
              (64, 56, 256, 1, 1), (256, 56, 64, 1, 1), (128, 28, 512, 1, 1), (1024, 14, 256, 1, 1)]
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
            res = {"on": [], "off": []}
            for _ in range(5):
                for mode in ("on", "off"):
                    C.gemm_f32_set_cvec(mode == "on")
                    res[mode].append(timeit(fn))
            C.gemm_f32_set_cvec(True)
            print(json.dumps({"shape": [Cin, H, Cout, R], "pass": tag,
                              "on_us": round(min(res["on"]), 1), "off_us": round(min(res["off"]), 1)}),
                  flush=True)


if __name__ == "__main__":
    main()
