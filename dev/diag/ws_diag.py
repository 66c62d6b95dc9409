"""Diagnose the warp-specialised wgrad+SGD kernel: one SGD step (no momentum) on a ToyMLP,
recover each weight's gradient from the update (p0 - p1) / lr, compare with torch autograd."""
import sys
import torch
sys.path.insert(0, ".")
import tutorial_torch_distributed_data_parallel_amd as tdp
from tutorial_torch_distributed_data_parallel_amd._native import native
from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP

tdp.init_process_group("nccl", rank=0, world_size=1, local_rank=0)
dims = (512, 384, 256)
for ws in (False, True):
    native().wgrad_opt_set_enabled(ws)
    torch.manual_seed(5)
    m = ToyMLP(in_features=dims[0], hidden=dims[1:], num_classes=10, device="cuda")
    ref = ToyMLP(in_features=dims[0], hidden=dims[1:], num_classes=10, device="cuda")
    ref.load_state_dict(m.state_dict())
    d = tdp.DDP(m, device_ids=[0])
    o = tdp.optim.SGD(d.parameters(), lr=1.0, momentum=0.0)
    d.register_fused_optimizer(o)
    p0 = [p.detach().clone() for p in m.parameters()]
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn(128, dims[0], device="cuda", generator=g)
    y = torch.randint(0, 10, (128,), device="cuda", generator=g)
    o.zero_grad(set_to_none=True)
    tdp.ops.cross_entropy(d(x), y).backward()
    o.step()
    torch.cuda.synchronize()
    out = torch.nn.functional.cross_entropy(ref(x.double() if False else x), y)
    out.backward()
    for (n, p), a, (_, q) in zip(m.named_parameters(), p0, ref.named_parameters()):
        gr = (a - p.detach()).double()
        err = (gr - q.grad.double()).abs()
        tol = 1e-6 + 1e-4 * q.grad.double().abs()
        bad = (err > tol).nonzero()
        print(f"ws={ws} {n} {tuple(p.shape)} max_err={err.max().item():.3e} bad={len(bad)}")
        if len(bad) and p.dim() == 1:
            print("  first:", [(round(float(gr[i]), 6), round(float(q.grad[i]), 6)) for i in range(6)])
            print("  ratio mean:", float((gr / q.grad.double()).mean()))
        if len(bad) and p.dim() == 2:
            r, c = bad[:, 0], bad[:, 1]
            print("  rows%128:", sorted(set((r % 128).tolist()))[:40])
            print("  cols%128:", sorted(set((c % 128).tolist()))[:40])
            print("  tiles:", sorted(set(((r // 128) * 1000 + c // 128).tolist()))[:40])
            print("  sample:", [(int(a_), int(b_), float(gr[a_, b_]), float(q.grad[a_, b_])) for a_, b_ in bad[:6].tolist()])
tdp.destroy_process_group()
