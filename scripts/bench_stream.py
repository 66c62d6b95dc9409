"""HBM streaming ceiling on this box: bytes/s of (a) torch copy, (b) the native flat SGD update
(p, g, momentum: 12 B read + 8 B written per element), (c) the fused wgrad+SGD epilogue GEMM of
the toy MLP's fc1 (p, momentum: 16 B per element + the GEMM), all over the toy-MLP parameter
count. The gap between (b)/(a) and (c) is what a streaming-optimal wgrad+optimizer kernel could
recover. python scripts/bench_stream.py"""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from tutorial_torch_distributed_data_parallel_amd._native import native  # noqa: E402

C = native()


def timeit(fn, reps=20):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps * 1000.0


x = torch.randn(4096, 4096, device="cuda")
for _ in range(40):
    torch.mm(x, x)
n = 9216 * 4096 + 4096 * 4096
a = torch.randn(n, device="cuda")
b = torch.empty_like(a)
us = timeit(lambda: b.copy_(a))
print(json.dumps({"copy": {"us": round(us, 1), "TBps": round(8 * n / us / 1e6, 2)}}))
p, g, m = torch.randn(n, device="cuda"), torch.randn(n, device="cuda"), torch.zeros(n, device="cuda")
us = timeit(lambda: C.sgd_flat(p, g, m, 1e-4, 0.9, 0.0, 0.0, False, False, False))
print(json.dumps({"sgd_flat": {"us": round(us, 1), "TBps": round(20 * n / us / 1e6, 2)}}))
# fc1 wgrad + SGD epilogue through a registered DDP (world 1): dW = g^T x, update p / momentum
import tutorial_torch_distributed_data_parallel_amd as tdp  # noqa: E402

tdp.init_process_group("nccl", rank=0, world_size=1, local_rank=0)
lin = tdp.nn.Linear(9216, 4096, device="cuda")
d = tdp.DDP(lin, device_ids=[0])
opt = tdp.optim.SGD(d.parameters(), lr=1e-4, momentum=0.9)
d.register_fused_optimizer(opt)
xb = torch.randn(128, 9216, device="cuda")
gy = torch.randn(128, 4096, device="cuda")


def step():
    opt.zero_grad(set_to_none=True)
    d(xb).backward(gy)


for _ in range(3):
    step()
us = timeit(step)
ne = 9216 * 4096
print(json.dumps({"fc1_wgrad_sgd_step_incl_fwd": {"us": round(us, 1)}}))
tdp.destroy_process_group()
