"""Diagnostic: the one-process Accelerate path (hidden world-1 DDP) against the native DDP step,
per step and per parameter, in three set-ups -- two native DDPs (control), native vs hidden with
the optimizer built before prepare (as the reference script does), native vs hidden with the
optimizer built after prepare -- and how many weight-gradient GEMMs took the optimizer
epilogue in each model. GPU only.

    python scripts/diag_accel_hidden.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import tutorial_torch_distributed_data_parallel_amd as tdp  # noqa: E402
from tutorial_torch_distributed_data_parallel_amd.accelerate import Accelerator  # noqa: E402
from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP  # noqa: E402
from tutorial_torch_distributed_data_parallel_amd.parallel.ddp import DistributedDataParallel  # noqa: E402

DIMS = dict(in_features=1024, hidden=(512, 512), num_classes=10)
EPI = {}
_orig = DistributedDataParallel.epilogue_slot


def _count(self, p):
    r = _orig(self, p)
    EPI[id(self)] = EPI.get(id(self), 0) + (r is not None)
    return r


DistributedDataParallel.epilogue_slot = _count


def build(kind, acc=None):
    torch.manual_seed(0)
    m = ToyMLP(**DIMS, device="cuda")
    if kind == "native":
        d = tdp.DDP(m, device_ids=[0])
        o = tdp.optim.SGD(d.parameters(), lr=0.05, momentum=0.9)
        assert d.register_fused_optimizer(o)
        return m, (lambda x: d(x)), o, o, d
    if kind == "hidden_opt_first":
        o = tdp.optim.SGD(m.parameters(), lr=0.05, momentum=0.9)
        model, opt = acc.prepare(m, o)
    else:
        model = acc.prepare(m)
        o = tdp.optim.SGD(model.parameters(), lr=0.05, momentum=0.9)
        opt = acc.prepare(o)
    assert acc.fuse_optimizer(model, opt)
    return m, model, opt, o, acc.ddp_of(model)


def main():
    tdp.init_process_group("nccl", rank=0, world_size=1, local_rank=0)
    g = torch.Generator(device="cuda").manual_seed(7)
    data = [(torch.randn(64, DIMS["in_features"], device="cuda", generator=g),
             torch.randint(0, 10, (64,), device="cuda", generator=g)) for _ in range(6)]
    for other in ("native", "hidden_opt_first", "hidden_opt_after"):
        acc = Accelerator()
        EPI.clear()
        m1, f1, s1, o1, d1 = build("native")
        m2, f2, s2, o2, d2 = build(other, acc)
        rows = []
        for i, (x, y) in enumerate(data):
            if i == 3:
                for o in (o1, o2):
                    o.param_groups[0]["lr"] *= 0.5
            for f, s in ((f1, s1), (f2, s2)):
                s.zero_grad(set_to_none=True)
                tdp.ops.backward(tdp.ops.cross_entropy(f(x), y))
                s.step()
            torch.cuda.synchronize()
            rows.append({n: float((a - b).abs().max())
                         for (n, a), b in zip(m1.named_parameters(), m2.parameters())})
        print(json.dumps({"vs": other, "epilogue_gemms": {"native": EPI.get(id(d1), 0),
                                                          other: EPI.get(id(d2), 0)},
                          "max_diff_per_step": rows}), flush=True)
    tdp.destroy_process_group()


if __name__ == "__main__":
    main()
