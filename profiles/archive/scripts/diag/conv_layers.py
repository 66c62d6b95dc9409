"""Per-layer check of every ResNet-50 / AlexNet conv shape: native fwd/dgrad/wgrad vs float64 CPU."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch
import torch.nn.functional as F

from tutorial_torch_distributed_data_parallel_amd import ops
from tutorial_torch_distributed_data_parallel_amd.models.registry import build_model

name = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
hw = int(sys.argv[2]) if len(sys.argv) > 2 else 64
n = int(sys.argv[3]) if len(sys.argv) > 3 else 8
m = build_model(name)
shapes = {}
hooks = []
for mn, mod in m.named_modules():
    if isinstance(mod, torch.nn.Conv2d):
        def hk(mod, inp, out, mn=mn):
            shapes.setdefault((tuple(inp[0].shape), tuple(mod.weight.shape), mod.stride,
                               mod.padding), mn)
        hooks.append(mod.register_forward_hook(hk))
with torch.no_grad():
    m.eval()(torch.randn(n, 3, hw, hw))
worst = 0
for (xs, ws, st, pd), mn in shapes.items():
    torch.manual_seed(0)
    x = torch.randn(xs, device="cuda", requires_grad=True)
    w = (torch.randn(ws, device="cuda") / (ws[1] * ws[2] * ws[3]) ** 0.5).requires_grad_()
    y = ops.conv2d(x, w, None, st, pd)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().double().cpu().requires_grad_()
    wr = w.detach().double().cpu().requires_grad_()
    yr = F.conv2d(xr, wr, None, st, pd)
    yr.backward(dy.double().cpu())

    def rel(a, b):
        return ((a.double().cpu() - b).abs().max() / (b.abs().max() + 1e-12)).item()
    e = (rel(y, yr), rel(x.grad, xr.grad), rel(w.grad, wr.grad))
    worst = max(worst, max(e))
    print(f"{mn:28s} x{list(xs)} w{list(ws)} s{st} p{pd}  fwd {e[0]:.2e} dgrad {e[1]:.2e} "
          f"wgrad {e[2]:.2e}", flush=True)
print("worst", worst)
