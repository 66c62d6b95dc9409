"""A few ResNet-50 conv GEMMs (forward / input grad / weight grad) for PMC passes:
python scripts/conv_pmc_probe.py  (5 launches of each, after 2 warm-up launches)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from tutorial_torch_distributed_data_parallel_amd import ops

CASES = [  # (tag, Cin, H, Cout, R, stride, pad)
    ("l1_3x3", 64, 56, 64, 3, 1, 1), ("l3_3x3", 256, 14, 256, 3, 1, 1),
    ("l1_ds1x1", 64, 56, 256, 1, 1, 0), ("l3_1x1in", 1024, 14, 256, 1, 1, 0)]
B = 128
for tag, Cin, H, Cout, R, st, pd in CASES:
    x = torch.randn(B, Cin, H, H, device="cuda").contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, R, R, device="cuda") * 0.05).contiguous(
        memory_format=torch.channels_last)
    xr = x.clone().requires_grad_()
    wr = w.clone().requires_grad_()
    y = ops.conv2d(xr, wr, None, st, pd)
    dy = torch.randn_like(y)
    for i in range(7):
        with torch.no_grad():
            ops.conv2d(x, w, None, st, pd)
        torch.autograd.grad(y, (xr, wr), dy, retain_graph=True)
    torch.cuda.synchronize()
    print(tag, "done", flush=True)
