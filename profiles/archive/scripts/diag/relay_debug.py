"""Debug: W ranks on one GPU (host relay); print arena layout, buckets and mismatching arena
ranges of each config against the fp32 oracle (tests/relay_workers.py)."""
import functools
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))

import torch  # noqa: E402

import relay_workers as RW  # noqa: E402
import tutorial_torch_distributed_data_parallel_amd as tdp  # noqa: E402
from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP  # noqa: E402
from tutorial_torch_distributed_data_parallel_amd.parallel import runtime as rt  # noqa: E402
from tutorial_torch_distributed_data_parallel_amd.parallel.launcher import spawn  # noqa: E402


def worker(rank, factor, fused, kind, steps, ragged, rebuild=True, rep=None):
    tdp.init_process_group("relay")
    r, W = rt.get_rank(), rt.get_world_size()
    torch.manual_seed(0)
    model = ToyMLP(**RW.DIMS, device="cuda")
    ref = RW._torch_mlp(model)
    ddp = tdp.DDP(model, device_ids=[rt.device().index], factor_sync=factor,
                  rebuild_buckets=rebuild)
    ddp.factor_replicate = rep
    opt, ropt = RW._opts(kind, ddp.parameters(), ref.parameters(), 0.05 if kind == "sgd" else 2e-3)
    if fused:
        ddp.register_fused_optimizer(opt)
    rr, rs = (W - 1, 4) if ragged else (-1, -1)
    for step in range(steps):
        x, y = RW._batch(r, step, rr, rs)
        opt.zero_grad(set_to_none=True)
        tdp.ops.cross_entropy(ddp(x), y).backward()
        opt.step()
        RW._oracle_step(ref, ropt, W, step, rr, rs)
        torch.cuda.synchronize()
        a = ddp.arena
        names = [n for n, _ in model.named_parameters()]
        bad = []
        for i, (p, q) in enumerate(zip(model.parameters(), ref.parameters())):
            d = (p.detach() - q.detach()).abs().flatten()
            tol = 5e-5 + 2e-4 * q.detach().abs().flatten()
            idx = (d > tol).nonzero().flatten()
            if len(idx):
                bad.append((names[i], int(idx.min()), int(idx.max()), len(idx), float(d.max())))
        # arena data across ranks: first differing element ranges
        allp = rt.all_gather_flat(a.data.clone()).view(W, -1)
        diff = (allp[0] != allp[1]).nonzero().flatten()
        rng = (int(diff.min()), int(diff.max()), len(diff)) if len(diff) else None
        if r == 0 or bad:
            print(f"[r{r}] step {step} factor={factor} fused={fused} rebuilt={ddp._rebuilt} "
                  f"bounds={ddp._bounds} arena_diff={rng} bad={bad}", flush=True)
    if r == 0:
        print(f"[r{r}] offsets={list(zip([n for n,_ in model.named_parameters()], ddp.arena.offsets))}"
              f" numels={ddp.arena.numels} bounds={ddp._bounds} plan={ddp.sync_plan()}", flush=True)
    tdp.destroy_process_group()


if __name__ == "__main__":
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    for factor, fused, kind, rebuild, rep in [(True, True, "sgd", True, True),
                                              (True, True, "sgd", False, True),
                                              (True, True, "sgd", True, False),
                                              (False, True, "sgd", True, None)]:
        print("CONFIG", factor, fused, kind, rebuild, rep, flush=True)
        try:
            spawn(functools.partial(worker, factor=factor, fused=fused, kind=kind, steps=3,
                                    ragged=False, rebuild=rebuild, rep=rep), W, grace=5.0)
        except Exception as e:  # noqa: BLE001
            print("FAILED", factor, fused, kind, str(e)[-500:])
