"""Weight-gradient plan sweep: orientation (dW vs dW^T) x tile width x split-K x pipeline depth.

python scripts/sweep_wgrad.py [alexnet|resnet50] [batch] [targets]
One JSON line per (layer, config) with microseconds; last line per layer = best config and the
auto plan's time. Calls the native kernel directly (no autograd, no weight re-layout).
"""
import itertools
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

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
    name = sys.argv[1] if len(sys.argv) > 1 else "alexnet"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    m = build_model(name)
    shapes = {}
    for mn, mod in m.named_modules():
        if isinstance(mod, torch.nn.Conv2d):
            mod.register_forward_hook(lambda mod, i, o, mn=mn: shapes.setdefault(
                (tuple(i[0].shape[1:]), tuple(mod.weight.shape), mod.stride, mod.padding),
                mn) and None)
    with torch.no_grad():
        m.eval()(torch.randn(1, 3, 224, 224))
    C = native()
    for (xs, ws, st, pd), mn in shapes.items():
        Cin, H, W = xs
        Cout, _, R, S = ws
        Cp = (Cin + 3) // 4 * 4
        P = (H + 2 * pd[0] - R) // st[0] + 1
        Q = (W + 2 * pd[1] - S) // st[1] + 1
        x = torch.randn(B, Cp, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
        dy = torch.randn(B, Cout, P, Q, device="cuda").contiguous(memory_format=torch.channels_last)
        dw = torch.empty(Cout * R * S * Cp, device="cuda")
        flops = 2.0 * B * P * Q * Cout * Cp * R * S
        run = lambda: C.conv_nhwc_wgrad(dy, x, dw, R, S, st[0], st[1], pd[0], pd[1], 0.0)
        C.conv_set_wgrad_transposed(-1)
        C.gemm_f32_set_override(0, 0, 0)
        t_auto = timeit(run)
        auto_t = C.conv_wgrad_transposed(Cout, R, S, Cp)
        best = (t_auto, "auto")
        if len(sys.argv) > 3 and sys.argv[3] == "targets":  # auto plan, split-K target per CU
            rec = {}
            for tg in (2, 3, 4, 5, 6, 8, 12):
                C.conv_set_wgrad_target(tg)
                rec[tg] = round(timeit(run), 1)
            C.conv_set_wgrad_target(0)
            print(json.dumps({"layer": mn, "w": list(ws), "x": [B, Cp, H, W], "auto_T": auto_t,
                              "target_us": rec}), flush=True)
            continue
        for tr, fn, sp, stg in itertools.product((0, 1), (1, 2), (0, 2, 4, 8, 16, 32), (0, 2, 3)):
            if fn == 2 and stg == 3:
                continue
            C.conv_set_wgrad_transposed(tr)
            C.gemm_f32_set_override(fn, sp, stg)
            t = timeit(run, iters=10, warm=2)
            cfg = f"T{tr}/fn{fn}/sp{sp}/st{stg}"
            print(json.dumps({"layer": mn, "cfg": cfg, "us": round(t, 1),
                              "tflops": round(flops / t / 1e6, 1)}), flush=True)
            if t < best[0]:
                best = (t, cfg)
        C.conv_set_wgrad_transposed(-1)
        C.gemm_f32_set_override(0, 0, 0)
        print(json.dumps({"layer": mn, "x": [B, Cp, H, W], "w": list(ws), "auto_T": auto_t,
                          "auto_us": round(t_auto, 1), "best": best[1],
                          "best_us": round(best[0], 1)}), flush=True)


if __name__ == "__main__":
    main()
