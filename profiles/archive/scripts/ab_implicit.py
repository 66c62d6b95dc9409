"""Implicit-GEMM operand overhead: a 1x1 stride-1 convolution (implicit A: per-chunk pixel/tap
address math) vs the same GEMM with a dense K-contiguous A, plus a 4096^3 dense GEMM for the
kernel's ceiling. One JSON line per shape (min of 5 runs of 20)."""
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
for (B, Cin, H, Cout) in [(128, 256, 56, 64), (128, 64, 56, 256), (128, 512, 28, 128),
                          (128, 1024, 14, 256), (128, 128, 28, 512)]:
    x = torch.randn(B, Cin, H, H, device="cuda").contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, 1, 1, device="cuda") * 0.05).contiguous(
        memory_format=torch.channels_last)
    A = x.permute(0, 2, 3, 1).reshape(-1, Cin)
    Wm = w.reshape(Cout, Cin)
    out = torch.empty(A.shape[0], Cout, device="cuda")
    conv = lambda: ops.conv2d(x, w, None, 1, 0)
    dense = lambda: C.gemm_f32(A, Wm, out, True, True)
    torch.testing.assert_close(conv().permute(0, 2, 3, 1).reshape(-1, Cout), (dense(), out)[1],
                               atol=1e-3, rtol=1e-3)
    tc = min(timeit(conv) for _ in range(5))
    td = min(timeit(dense) for _ in range(5))
    fl = 2.0 * A.shape[0] * Cin * Cout
    print(json.dumps({"M": A.shape[0], "K": Cin, "N": Cout, "implicit_us": round(tc, 1),
                      "dense_us": round(td, 1), "implicit_tf": round(fl / tc / 1e6, 1),
                      "dense_tf": round(fl / td / 1e6, 1)}), flush=True)
for n in (4096, 8192):
    A = torch.randn(n, n, device="cuda")
    Bm = torch.randn(n, n, device="cuda")
    out = torch.empty(n, n, device="cuda")
    for ak, bk in ((True, True), (True, False), (False, False)):
        t = min(timeit(lambda: C.gemm_f32(A, Bm, out, ak, bk), iters=5) for _ in range(3))
        print(json.dumps({"square": n, "a_k": ak, "b_k": bk, "us": round(t, 1),
                          "tf": round(2.0 * n ** 3 / t / 1e6, 1)}), flush=True)
