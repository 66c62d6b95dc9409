"""Forward / input-gradient plan sweep (tile width x pipeline depth) per conv shape.

python scripts/sweep_conv_fd.py [alexnet|resnet50] [batch]
One JSON line per layer: microseconds of the native forward and stride-1 input-gradient kernels
under the auto plan and every (FN, stages) override.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from tutorial_torch_distributed_data_parallel_amd._native import native
from tutorial_torch_distributed_data_parallel_amd.models.registry import build_model

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from sweep_wgrad import timeit  # noqa: E402


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
    cfgs = [(0, 0), (1, 2), (1, 3), (2, 2)]
    for (xs, ws, st, pd), mn in shapes.items():
        Cin, H, W = xs
        Cout, _, R, S = ws
        Cp = (Cin + 3) // 4 * 4
        P = (H + 2 * pd[0] - R) // st[0] + 1
        Q = (W + 2 * pd[1] - S) // st[1] + 1
        x = torch.randn(B, Cp, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
        wt = torch.randn(Cout, R, S, Cp, device="cuda") * 0.05
        dy = torch.randn(B, Cout, P, Q, device="cuda").contiguous(memory_format=torch.channels_last)
        w2 = torch.randn(R, S, Cout, Cp, device="cuda") * 0.05
        rec = {"layer": name + ":" + mn, "x": [B, Cp, H, W], "w": list(ws), "stride": st[0]}
        for tag, run in (
                ("fwd", lambda: C.conv_nhwc_fwd(x, wt, None, R, S, st[0], st[1], pd[0], pd[1],
                                                False)),
                ("dgrad", (lambda: C.conv_nhwc_dgrad(dy, w2, list(x.shape), R, S, 1, 1, pd[0],
                                                     pd[1])) if st == (1, 1) else None)):
            if run is None:
                continue
            res = {}
            for fn, stg in cfgs:
                C.gemm_f32_set_override(fn, 0, stg)
                res[f"fn{fn}/st{stg}"] = round(timeit(run), 1)
            C.gemm_f32_set_override(0, 0, 0)
            rec[tag] = res
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
