"""Per-rank compute of the tensor-sharded toy-MLP step at W ranks, on ONE GPU: the process plays
rank 0 with the shard shapes of a W-rank job and every collective replaced by its local copy
(parallel/tensor_parallel.py set_fake_world). Captured step (as bench.py runs it), SGD momentum,
B = 128 per rank. Prints one JSON line per W: ms per step of the rank's compute, next to the dp1
step of the replicated model measured the same way. The W-rank step is this plus the exposed
part of its collectives (docs/COMM_MODEL.md "Tensor-sharded").

python scripts/tp_rank_proxy.py [W ...]"""
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
import tutorial_torch_distributed_data_parallel_amd as tdp  # noqa: E402
from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP  # noqa: E402
from tutorial_torch_distributed_data_parallel_amd.parallel import tensor_parallel as TPm  # noqa
from tutorial_torch_distributed_data_parallel_amd.train.graph import CapturedStep  # noqa: E402

tdp.init_process_group("nccl", rank=0, world_size=1, local_rank=0)
dev = torch.device("cuda", 0)
B = 128


def timed(step, n=200):
    g = CapturedStep(step, warmup=3)
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1000.0 / n


def run(W):
    TPm.set_fake_world(W)
    torch.manual_seed(0)
    m = ToyMLP(device=dev)
    # the bench's form: every rank gathers the node's batch itself (no input all-gather)
    net = TPm.TensorParallelMLP(m, global_batch=True) if W > 0 else tdp.DDP(m, device_ids=[0])
    opt = tdp.optim.SGD(net.parameters(), lr=0.01, momentum=0.9)
    if W == 0:
        net.register_fused_optimizer(opt)
    x = torch.randn(B * max(W, 1), 9216, device=dev)
    y = torch.randint(0, 10, (B,), device=dev)

    def step():
        opt.zero_grad(set_to_none=True)
        tdp.ops.backward(tdp.ops.cross_entropy(net(x), y))
        if W > 0:
            net.sync_grads()
        opt.step()
    ms = timed(step)
    TPm.set_fake_world(0)
    return ms


# clock warm-up
a = torch.randn(4096, 4096, device=dev)
for _ in range(50):
    a @ a
torch.cuda.synchronize()
args = [v for v in sys.argv[1:] if v != "--no-dp1"]
ws = [int(v) for v in args] or [1, 2, 4, 8]
if "--no-dp1" not in sys.argv:
    print(json.dumps({"W": "dp1 (DDP, fused optimizer)", "ms": round(run(0), 4)}), flush=True)
for W in ws:
    print(json.dumps({"W": W, "rank_compute_ms": round(run(W), 4)}), flush=True)
