"""Time the toy MLP's fc1 / fc2 weight-gradient + SGD kernels alone (world-size-1 DDP, fused
SGD in the GEMM epilogue): run under rocprofv3 --kernel-trace; TDP_WS_EXP / TDP_WGRAD_WS pick
variants. python dev/micro/ws_probe.py [steps]"""
import sys

import torch

sys.path.insert(0, ".")
import tutorial_torch_distributed_data_parallel_amd as tdp  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
tdp.init_process_group("nccl", rank=0, world_size=1, local_rank=0)
for (o, i) in ((4096, 9216), (4096, 4096)):
    lin = tdp.nn.Linear(i, o, device="cuda")
    d = tdp.DDP(lin, device_ids=[0])
    opt = tdp.optim.SGD(d.parameters(), lr=1e-4, momentum=0.9)
    d.register_fused_optimizer(opt)
    xb = torch.randn(128, i, device="cuda")
    gy = torch.randn(128, o, device="cuda")
    for _ in range(steps):
        opt.zero_grad(set_to_none=True)
        d(xb).backward(gy)
    torch.cuda.synchronize()
    del lin, d, opt
tdp.destroy_process_group()
