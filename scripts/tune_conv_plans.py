"""Measure every (tile width FN, split-K) plan of each convolution pass and write the winners to
the plan table (ops/plan_db.py).

python scripts/tune_conv_plans.py OUT.json resnet50:128 alexnet:128 ...
For every unique convolution of the models (at that per-GPU batch) and every pass (forward,
input gradient, weight gradient), time the heuristic plan and each candidate override
(interleaved, min of 3 x 10 launches). Keep a candidate only when it beats the heuristic by
>= 3 %. One JSON line per (layer, pass) goes to stdout. The table (with the measured
microseconds) goes to OUT.json.
"""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from tutorial_torch_distributed_data_parallel_amd import ops
from tutorial_torch_distributed_data_parallel_amd._native import native
from tutorial_torch_distributed_data_parallel_amd.models.registry import build_model



def timeit(fn, iters=20):
    """us per call of ``fn`` (device events, one untimed call first)."""
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / iters

FD = [(fn, s) for fn in (1, 2) for s in (1, 2, 3, 4, 6, 8)]


def wgrad_candidates(M, N, K, cus=256):
    out = []
    for fn in (1, 2):
        tiles = math.ceil(M / 128) * math.ceil(N / (64 * fn))
        kmax = max(1, K // (32 * 8))
        for per_cu in (1, 2, 3, 4, 6, 8, 12, 16):
            s = min(kmax, max(1, math.ceil(per_cu * cus / tiles)))
            if (fn, s) not in out:
                out.append((fn, s))
    return out


def conv_shapes(name, B):
    m = build_model(name)
    shapes = {}
    for mn, mod in m.named_modules():
        if isinstance(mod, torch.nn.Conv2d):
            def hook(mod, i, o, mn=mn):
                shapes.setdefault((tuple(i[0].shape[1:]), tuple(mod.weight.shape), mod.stride,
                                   mod.padding), mn)
            mod.register_forward_hook(hook)
    with torch.no_grad():
        m.eval()(torch.randn(1, 3, 224, 224))
    return [((B,) + xs, ws, st, pd, mn) for (xs, ws, st, pd), mn in shapes.items()]


def main():
    out_path = sys.argv[1]
    C = native()
    C.conv_plan_db_clear()
    os.environ["TDP_CONV_PLAN_DB"] = "0"  # measure against the heuristic alone
    plans = []
    for spec in sys.argv[2:]:
        name, B = spec.split(":")
        for xs, ws, st, pd, mn in conv_shapes(name, int(B)):
            x = torch.randn(xs, device="cuda").contiguous(memory_format=torch.channels_last)
            w = torch.randn(ws, device="cuda") * 0.05
            if xs[1] % 4 == 0:
                w = w.contiguous(memory_format=torch.channels_last)
            xr = x.clone().requires_grad_()
            wr = w.clone().requires_grad_()
            y_x = ops.conv2d(xr, w, None, st, pd)
            y_w = ops.conv2d(x, wr, None, st, pd)
            dy = torch.randn_like(y_x)
            Cout, Cin, R, S = ws
            P, Q = y_x.shape[2], y_x.shape[3]
            def fwd_bn():
                # ResNet: a BatchNorm follows -- an unsplit plan's epilogue emits its statistics,
                # a split plan leaves a moments pass over the output (price both)
                y = ops.conv2d(x, w, None, st, pd, bn_stats=True)
                tag = getattr(y, "_tdp_bn_part", None)
                if tag is None:
                    C.bn_moments(y.permute(0, 2, 3, 1).reshape(-1, y.shape[1]))
                else:
                    C.bn_moments_partials(tag[0], float(y.numel() // y.shape[1]))

            fwd = fwd_bn if name == "resnet50" else (lambda: ops.conv2d(x, w, None, st, pd))
            passes = [("fwd", fwd, FD),
                      ("wgrad", lambda: torch.autograd.grad(y_w, wr, dy, retain_graph=True),
                       wgrad_candidates(Cout, R * S * ((Cin + 3) // 4 * 4), xs[0] * P * Q))]
            if xs[1] >= 4:  # the stem's input needs no gradient
                passes.insert(1, ("dgrad", lambda: torch.autograd.grad(y_x, xr, dy,
                                                                       retain_graph=True), FD))
            for tag, fn, cands in passes:
                res = {}
                for _ in range(3):
                    for f, s in [(0, 0)] + cands:
                        C.gemm_f32_set_override(f, s, 0)
                        res.setdefault((f, s), []).append(timeit(fn, iters=10))
                C.gemm_f32_set_override(0, 0, 0)
                t = {k: min(v) for k, v in res.items()}
                best = min(t, key=t.get)
                rec = {"model": name, "layer": mn, "pass": tag, "x": list(xs), "w": list(ws),
                       "stride": list(st), "padding": list(pd), "auto_us": round(t[(0, 0)], 1),
                       "best": list(best), "best_us": round(t[best], 1)}
                print(json.dumps(rec), flush=True)
                if best != (0, 0) and t[best] < 0.97 * t[(0, 0)]:
                    plans.append({"pass": tag, "x": list(xs), "w": list(ws), "stride": list(st),
                                  "padding": list(pd), "fn": best[0], "splits": best[1],
                                  "us_heuristic": round(t[(0, 0)], 1), "us": round(t[best], 1),
                                  "model": name, "layer": mn})
    with open(out_path, "w") as f:
        json.dump({"device": "gfx950 (MI355X)", "tool": "scripts/tune_conv_plans.py",
                   "plans": plans}, f, indent=1)


if __name__ == "__main__":
    main()
