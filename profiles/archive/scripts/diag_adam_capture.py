"""Diagnostic: the captured-Adam-with-LR-change step (tests/test_sync_gpu.py
test_captured_adam_with_lr_change_matches_eager) repeated in ONE process with several seeds;
for every run prints the max / count of parameter differences between the eager and the
replayed model per parameter and, where they differ, the 128 x 128 tiles that hold the
differences -- to tell a summation-order difference (scattered, every run) from a race
(tile-shaped, some runs). GPU only.

    python scripts/diag_adam_capture.py --runs 8
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import tutorial_torch_distributed_data_parallel_amd as tdp  # noqa: E402
from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP  # noqa: E402
from tutorial_torch_distributed_data_parallel_amd.train.graph import CapturedStep  # noqa: E402


def one(seed: int, fused: bool) -> dict:
    def build():
        torch.manual_seed(3)
        m = ToyMLP(in_features=512, hidden=(512, 256), num_classes=10, device="cuda")
        d = tdp.DDP(m, device_ids=[0])
        o = tdp.optim.Adam(d.parameters(), lr=2e-3)
        if fused:
            assert d.register_fused_optimizer(o)
        return m, d, o

    g = torch.Generator(device="cuda").manual_seed(seed)
    X = torch.randn(1024, 512, device="cuda", generator=g)
    Y = torch.randint(0, 10, (1024,), device="cuda", generator=g)
    idx = torch.zeros(128, dtype=torch.long, device="cuda")

    def make_step(d, opt):
        def step():
            x, y = X.index_select(0, idx), Y.index_select(0, idx)
            opt.zero_grad(set_to_none=True)
            loss = tdp.ops.cross_entropy(d(x), y)
            loss.backward()
            opt.step()
            return loss
        return step

    m1, d1, o1 = build()
    m2, d2, o2 = build()
    eager = make_step(d1, o1)
    orders = [torch.randperm(1024, device="cuda", generator=g)[:128] for _ in range(13)]
    idx.copy_(orders[0])
    for _ in range(3):
        eager()
    graph = CapturedStep(make_step(d2, o2), warmup=3)
    loss_diff = 0.0
    for i, o in enumerate(orders[1:]):
        if i == 6:
            for opt in (o1, o2):
                opt.param_groups[0]["lr"] *= 0.25
        idx.copy_(o)
        le = eager()
        lg = graph.replay()
        loss_diff = max(loss_diff, float((le - lg).abs()))
    torch.cuda.synchronize()
    out = {"seed": seed, "fused": fused, "loss_max_diff": loss_diff, "params": {}}
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        d = (a.detach() - b.detach()).abs()
        rec = {"max": float(d.max()), "n_diff": int((d > 0).sum()),
               "n_over_1e-5": int((d > 1e-5).sum())}
        if d.dim() == 2 and rec["n_over_1e-5"]:
            r, c = torch.nonzero(d > 1e-5, as_tuple=True)
            tiles = torch.unique((r // 128) * 1000 + (c // 128)).tolist()
            rec["tiles_rc"] = [(t // 1000, t % 1000) for t in tiles][:16]
        out["params"][n] = rec
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=8)
    a = ap.parse_args()
    tdp.init_process_group("nccl", rank=0, world_size=1, local_rank=0)
    for s in range(a.runs):
        for fused in (True, False):
            print(json.dumps(one(s, fused)), flush=True)
    tdp.destroy_process_group()


if __name__ == "__main__":
    main()
