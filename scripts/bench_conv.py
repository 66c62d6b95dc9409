"""Per-layer conv timing: native NHWC implicit GEMM vs MIOpen (torch, NCHW and channels_last).

python scripts/bench_conv.py [resnet50|alexnet] [batch]
Prints one JSON line per unique conv shape with fwd / dgrad / wgrad microseconds and TFLOP/s.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

from tutorial_torch_distributed_data_parallel_amd._native import native
from tutorial_torch_distributed_data_parallel_amd.models.registry import build_model


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


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    m = build_model(name)
    shapes = {}
    for mn, mod in m.named_modules():
        if isinstance(mod, torch.nn.Conv2d):
            mod.register_forward_hook(lambda mod, i, o, mn=mn: shapes.setdefault(
                (tuple(i[0].shape[1:]), tuple(mod.weight.shape), mod.stride, mod.padding),
                [mn, 0]).__setitem__(1, shapes[(tuple(i[0].shape[1:]), tuple(mod.weight.shape),
                                                 mod.stride, mod.padding)][1] + 1))
    with torch.no_grad():
        m.eval()(torch.randn(1, 3, 224, 224))
    C = native()
    tot = {"ours": 0.0, "miopen_cl": 0.0, "miopen": 0.0}
    for (xs, ws, st, pd), (mn, cnt) in shapes.items():
        Cin, H, W = xs
        Cout, _, R, S = ws
        x = torch.randn(B, Cin, H, W, device="cuda")
        w = torch.randn(ws, device="cuda") * 0.05
        if Cin % 4 == 0:  # the Conv2d module's parameter layout (nn/modules.py)
            w = w.contiguous(memory_format=torch.channels_last)
        P = (H + 2 * pd[0] - R) // st[0] + 1
        Q = (W + 2 * pd[1] - S) // st[1] + 1
        flops = 2.0 * B * P * Q * Cout * Cin * R * S
        rec = {"layer": mn, "count": cnt, "x": [B, Cin, H, W], "w": list(ws), "stride": st[0],
               "gflop": round(flops / 1e9, 2)}
        from tutorial_torch_distributed_data_parallel_amd import ops

        xcl = x.contiguous(memory_format=torch.channels_last)
        dy = torch.randn(B, Cout, P, Q, device="cuda").contiguous(memory_format=torch.channels_last)
        with torch.no_grad():
            t_f = timeit(lambda: ops.conv2d(xcl, w, None, st, pd))
        # dgrad / wgrad through the autograd op (includes the weight re-layout copies, phase
        # decomposition and transposed-wgrad paths exactly as training runs them)
        xr = xcl.detach().clone().requires_grad_()
        wr = w.detach().clone().requires_grad_()
        y_x = ops.conv2d(xr, w, None, st, pd)
        y_w = ops.conv2d(xcl, wr, None, st, pd)
        t_d = timeit(lambda: torch.autograd.grad(y_x, xr, dy, retain_graph=True))
        t_w = timeit(lambda: torch.autograd.grad(y_w, wr, dy, retain_graph=True))
        rec["ours_us"] = [round(t_f, 1), round(t_d, 1), round(t_w, 1)]
        for tag, fmt in (("miopen", torch.contiguous_format), ("miopen_cl", torch.channels_last)):
            xx = x.contiguous(memory_format=fmt)
            ww = w.contiguous(memory_format=fmt)
            dd = dy.contiguous(memory_format=fmt)
            tf = timeit(lambda: F.conv2d(xx, ww, None, st, pd))
            td = timeit(lambda: torch.ops.aten.convolution_backward(
                dd, xx, ww, None, st, pd, (1, 1), False, (0, 0), 1, (True, False, False)))
            tw = timeit(lambda: torch.ops.aten.convolution_backward(
                dd, xx, ww, None, st, pd, (1, 1), False, (0, 0), 1, (False, True, False)))
            rec[tag + "_us"] = [round(tf, 1), round(td, 1), round(tw, 1)]
            tot[tag] += cnt * (tf + td + tw)
        tot["ours"] += cnt * (t_f + t_d + t_w)
        rec["ours_tflops"] = [round(flops / t / 1e6, 1) for t in (t_f, t_d, t_w)]
        print(json.dumps(rec), flush=True)
    print(json.dumps({"total_ms_per_step": {k: round(v / 1000, 2) for k, v in tot.items()}}))


if __name__ == "__main__":
    main()
