"""Forward / input-gradient plan sweep over (tile width FN, split-K) per conv shape, with the
planner's own choice for reference. The wave-quantisation question: a grid of T tiles on
3 (FN 1) or 2 (FN 2) workgroups per CU runs ceil(T / slots) rounds.

python scripts/sweep_fd_splits.py [resnet50|alexnet] [batch]  -> one JSON line per (layer, pass)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from tutorial_torch_distributed_data_parallel_amd import ops
from tutorial_torch_distributed_data_parallel_amd._native import native
from tutorial_torch_distributed_data_parallel_amd.models.registry import build_model

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ab_cvec import timeit  # noqa: E402

PLANS = [(0, 0)] + [(fn, s) for fn in (1, 2) for s in (1, 2, 3, 4, 6, 8)]


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    m = build_model(name)
    shapes = {}
    for mn, mod in m.named_modules():
        if isinstance(mod, torch.nn.Conv2d):
            def hook(mod, i, o, mn=mn):  # returns None: a hook's return value replaces the output
                shapes.setdefault((tuple(i[0].shape[1:]), tuple(mod.weight.shape), mod.stride,
                                   mod.padding), mn)
            mod.register_forward_hook(hook)
    with torch.no_grad():
        m.eval()(torch.randn(1, 3, 224, 224))
    C = native()
    for (xs, ws, st, pd), mn in shapes.items():
        Cin, H, W = xs
        if Cin % 4:
            continue  # the stem: its own path
        x = torch.randn(B, *xs, device="cuda").contiguous(memory_format=torch.channels_last)
        w = (torch.randn(ws, device="cuda") * 0.05).contiguous(memory_format=torch.channels_last)
        xr = x.clone().requires_grad_()
        y = ops.conv2d(xr, w, None, st, pd)
        dy = torch.randn_like(y)
        fwd = lambda: ops.conv2d(x, w, None, st, pd)
        dgr = lambda: torch.autograd.grad(y, xr, dy, retain_graph=True)
        for tag, fn in (("fwd", fwd), ("dgrad", dgr)):
            res = {}
            for _ in range(3):
                for f, s in PLANS:
                    C.gemm_f32_set_override(f, s, 0)
                    res.setdefault(f"{f}x{s}", []).append(timeit(fn, iters=10))
            C.gemm_f32_set_override(0, 0, 0)
            best = min(res, key=lambda k: min(res[k]))
            print(json.dumps({"layer": mn, "pass": tag, "x": [B, *xs], "w": list(ws),
                              "stride": st[0], "best": best,
                              **{k: round(min(v), 1) for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
