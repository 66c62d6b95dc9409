"""Per-step GPU time of the flagship bench step (toy MLP dp1): events around every step for the
first 300 steps of a fresh process, printed in groups of 10. Shows how many steps the device
needs before the step time settles (clock / power ramp, allocator, first-touch)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tutorial_torch_distributed_data_parallel_amd as tdp  # noqa: E402
from tutorial_torch_distributed_data_parallel_amd.data import SyntheticDataset  # noqa: E402
from tutorial_torch_distributed_data_parallel_amd.data.synthetic import gather_batch  # noqa: E402
from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP  # noqa: E402


def main():
    tdp.init_process_group("nccl")
    dev = tdp.parallel.runtime.device()
    torch.manual_seed(0)
    model = ToyMLP(in_features=9216, hidden=(4096, 4096), device=dev)
    ddp = tdp.DDP(model, device_ids=[dev.index])
    opt = tdp.optim.SGD(ddp.parameters(), lr=0.01, momentum=0.9)
    ddp.register_fused_optimizer(opt)
    data = SyntheticDataset(8192, (9216,), 10, seed=0, device=dev)
    idx = torch.randperm(8192, device=dev)
    acc = torch.zeros(3, device=dev)

    def step(i):
        b = idx[(i * 128) % 8192: (i * 128) % 8192 + 128]
        x, y = gather_batch(data.x, data.y, b)
        opt.zero_grad(set_to_none=True)
        tdp.ops.backward(tdp.ops.cross_entropy(ddp(x), y, acc=acc))
        opt.step()

    n = 300
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev[0].record()
    for i in range(n):
        step(i)
        ev[i + 1].record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1000
    ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(n)]
    for g in range(0, n, 10):
        seg = ms[g:g + 10]
        print(f"steps {g:3d}-{g + 9:3d}: mean {sum(seg) / len(seg):.4f} ms  min {min(seg):.4f}  "
              f"max {max(seg):.4f}")
    print(f"wall {wall:.1f} ms for {n} steps")
    tdp.destroy_process_group()


if __name__ == "__main__":
    main()
