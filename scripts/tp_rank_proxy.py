"""Per-rank compute of the tensor-sharded toy-MLP step at W ranks, on ONE GPU
(parallel/tensor_parallel.py ``rank_compute_ms``: rank 0's shard shapes, collectives as local
copies, captured step, the node's batch gathered per step), next to the captured dp1 step of the
replicated model (DDP, fused optimizer). One JSON line each.

python scripts/tp_rank_proxy.py [--no-dp1] [--unfused] [W ...]"""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
import tutorial_torch_distributed_data_parallel_amd as tdp  # noqa: E402
from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP  # noqa: E402
from tutorial_torch_distributed_data_parallel_amd.parallel.tensor_parallel import \
    rank_compute_ms  # noqa: E402
from tutorial_torch_distributed_data_parallel_amd.train.graph import CapturedStep  # noqa: E402

tdp.init_process_group("nccl", rank=0, world_size=1, local_rank=0)
dev = torch.device("cuda", 0)
B = 128


def dp1_ms(n=200):
    import time

    torch.manual_seed(0)
    m = ToyMLP(device=dev)
    ddp = tdp.DDP(m, device_ids=[0])
    opt = tdp.optim.SGD(ddp.parameters(), lr=0.01, momentum=0.9)
    ddp.register_fused_optimizer(opt)
    x = torch.randn(B, 9216, device=dev)
    y = torch.randint(0, 10, (B,), device=dev)

    def step():
        opt.zero_grad(set_to_none=True)
        tdp.ops.backward(tdp.ops.cross_entropy(ddp(x), y))
        opt.step()
    g = CapturedStep(step, warmup=3)
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1000.0 / n


a = torch.randn(4096, 4096, device=dev)  # clock warm-up
for _ in range(50):
    a @ a
torch.cuda.synchronize()
args = [v for v in sys.argv[1:] if v not in ("--no-dp1", "--unfused")]
FUSED = "--unfused" not in sys.argv
ws = [int(v) for v in args] or [1, 2, 4, 8]
if "--no-dp1" not in sys.argv:
    print(json.dumps({"W": "dp1 (DDP, fused optimizer)", "ms": round(dp1_ms(), 4)}), flush=True)
for W in ws:
    print(json.dumps({"W": W, "fused": FUSED,
                      "rank_compute_ms": round(rank_compute_ms(W, steps=200, fused=FUSED), 4)}),
          flush=True)
