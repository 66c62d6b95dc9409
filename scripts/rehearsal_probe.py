"""One-GPU rehearsal of the W > 1 DDP schedule, alone (for rocprofv3 kernel traces).

    python scripts/rehearsal_probe.py [--steps 200] [--skip-collectives] [--dp1]

Builds what bench.py's ``build_rehearsal`` builds (the headline toy MLP, DDP with
``force_collective=True`` and the fused optimizer: factored jobs, buckets, side-stream forks and
one-rank RCCL collectives), captures one training step into a hipGraph and replays it; prints
ms/step. ``--dp1`` runs the world-size-1 step instead (optimizer in the weight-gradient GEMM
epilogues), ``--skip-collectives`` turns the one-rank collectives into no-ops (the schedule
alone). Under ``rocprofv3 --kernel-trace`` the steady state is ``scripts/step_kernels.py <csv>
ce_fwd``."""
from __future__ import annotations

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--skip-collectives", action="store_true")
    ap.add_argument("--dp1", action="store_true")
    ap.add_argument("--opt-variant", type=int, default=None,
                    help="SGD epilogue flags for gemm_f32_set_opt_variant (A/B: 24 = LDS + "
                         "non-temporal, the default; 88 = + kOptPre)")
    a = ap.parse_args()
    import torch

    import tutorial_torch_distributed_data_parallel_amd as tdp
    from tutorial_torch_distributed_data_parallel_amd.data.synthetic import gather_batch
    from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP
    from tutorial_torch_distributed_data_parallel_amd.parallel import runtime as rt
    from tutorial_torch_distributed_data_parallel_amd.train.graph import CapturedStep

    if a.opt_variant is not None:
        from tutorial_torch_distributed_data_parallel_amd._native import native

        native().gemm_f32_set_opt_variant(a.opt_variant, -1, -1, 0)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    tdp.init_process_group("nccl", rank=0, world_size=1, local_rank=0)
    dev = rt.device()
    torch.manual_seed(0)
    m = ToyMLP(in_features=9216, hidden=(4096, 4096), device=dev)
    ddp = tdp.DDP(m, device_ids=[dev.index], force_collective=not a.dp1)
    opt = tdp.optim.SGD(ddp.parameters(), lr=0.01, momentum=0.9)
    ddp.register_fused_optimizer(opt)
    x = torch.randn(4096, 9216, device=dev)
    y = torch.randint(0, 10, (4096,), device=dev)
    idx = torch.randperm(4096, device=dev)[:128].contiguous()
    acc = torch.zeros(3, device=dev)

    def step():
        xb, yb = gather_batch(x, y, idx)
        opt.zero_grad(set_to_none=True)
        tdp.ops.backward(tdp.ops.cross_entropy(ddp(xb), yb, acc=acc))
        opt.step()

    if a.skip_collectives and ddp._ops is not None:
        ddp._ops.skip_collectives = True
    g = CapturedStep(step, warmup=3)
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        g.replay()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1000.0 / a.steps
    print(f"{'dp1' if a.dp1 else 'rehearsal'}{' (no collectives)' if a.skip_collectives else ''}"
          f"{'' if a.opt_variant is None else f' opt_variant {a.opt_variant}'}"
          f": {ms:.4f} ms/step, buckets {len(ddp._bounds) - 1}, plan {ddp.sync_plan()}",
          flush=True)
    tdp.destroy_process_group()


if __name__ == "__main__":
    main()
