"""Worker functions for the multi-process (gloo, CPU) tests; run under parallel.launcher.spawn."""
import os

import torch
import torch.distributed as dist

import tutorial_torch_distributed_data_parallel_amd as tdp
from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP
from tutorial_torch_distributed_data_parallel_amd.parallel import runtime as rt


def _init():
    tdp.init_process_group("gloo")
    return rt.get_rank(), rt.get_world_size()


def _gather(obj):
    out = [None] * rt.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def ddp_oracles(rank, out_dir):
    r, ws = _init()
    torch.manual_seed(100 + r)  # different local init on every rank
    model = ToyMLP(in_features=24, hidden=(16, 16), num_classes=5)
    local_init = [p.detach().clone() for p in model.parameters()]
    ddp = tdp.DDP(model, bucket_cap_mb=0.0005, split_bucket_mb=0.0003)
    # oracle 1: every rank now holds rank 0's parameters
    params = [p.detach().clone() for p in model.parameters()]
    allp = _gather(params)
    for other in allp:
        for a, b in zip(other, allp[0]):
            assert torch.equal(a, b)
    if r == 1:
        assert any(not torch.equal(a, b) for a, b in zip(local_init, params))
    # oracle 2: grad == mean of local grads
    ref = ToyMLP(in_features=24, hidden=(16, 16), num_classes=5)
    ref.load_state_dict(model.state_dict())
    g = torch.Generator().manual_seed(7 + r)
    x = torch.randn(8, 24, generator=g)
    y = torch.randint(0, 5, (8,), generator=g)
    tdp.ops.cross_entropy(ddp(x), y).backward()
    torch.nn.functional.cross_entropy(ref(x), y).backward()
    local = [p.grad.detach().clone() for p in ref.parameters()]
    all_local = _gather(local)
    mean = [sum(gs) / ws for gs in zip(*all_local)]
    for p, m in zip(model.parameters(), mean):
        torch.testing.assert_close(p.grad, m, atol=1e-6, rtol=1e-5)
    # gradients are views of the arena (zero-copy buckets)
    for i in range(len(ddp.arena.params)):
        assert ddp.arena.is_arena_grad(i)
    info = ddp._get_ddp_logging_data()
    assert info["num_buckets"] > 2
    # oracle 3: no_sync keeps local gradients and accumulates
    for p in model.parameters():
        p.grad = None
    with ddp.no_sync():
        tdp.ops.cross_entropy(ddp(x), y).backward()
    for p, lg in zip(model.parameters(), local):
        torch.testing.assert_close(p.grad, lg, atol=1e-6, rtol=1e-5)
    tdp.ops.cross_entropy(ddp(x), y).backward()  # synced: mean over ranks of (local + local)
    for p, m in zip(model.parameters(), mean):
        torch.testing.assert_close(p.grad, 2 * m, atol=1e-5, rtol=1e-4)
    all_acc = _gather([p.grad.detach().clone() for p in model.parameters()])
    for gs in zip(*all_acc):
        for gg in gs:
            torch.testing.assert_close(gg, gs[0], atol=1e-6, rtol=1e-5)
    # optimizer step keeps replicas identical
    opt = tdp.optim.SGD(ddp.parameters(), lr=0.1, momentum=0.9)
    for _ in range(3):
        opt.zero_grad()
        tdp.ops.cross_entropy(ddp(x), y).backward()
        opt.step()
    allp = _gather([p.detach().clone() for p in model.parameters()])
    for other in allp:
        for a, b in zip(other, allp[0]):
            assert torch.equal(a, b)
    tdp.destroy_process_group()


def syncbn_parity(rank, out_dir):
    r, ws = _init()
    torch.manual_seed(0)
    model = ToyMLP(in_features=12, hidden=(10,), num_classes=3, batchnorm=True)
    ref = ToyMLP(in_features=12, hidden=(10,), num_classes=3, batchnorm=True)
    ref.load_state_dict(model.state_dict())
    model = tdp.nn.convert_sync_batchnorm(model)
    ddp = tdp.DDP(model)
    g = torch.Generator().manual_seed(3)
    X = torch.randn(16, 12, generator=g) * 2 + 1
    Y = torch.randint(0, 3, (16,), generator=g)
    per = 16 // ws
    xs, ys = X[r * per:(r + 1) * per], Y[r * per:(r + 1) * per]
    out = ddp(xs)
    loss = tdp.ops.cross_entropy(out, ys, reduction="sum")
    loss.backward()
    # reference: one process, full batch, plain BN; DDP averages grads -> compare to grad/ws
    rout = ref(X)
    torch.nn.functional.cross_entropy(rout, Y, reduction="sum").backward()
    torch.testing.assert_close(out, rout[r * per:(r + 1) * per].detach(), atol=1e-5, rtol=1e-5)
    for (n, p), (rn, rp) in zip(model.named_parameters(), ref.named_parameters()):
        torch.testing.assert_close(p.grad * ws, rp.grad, atol=1e-4, rtol=1e-4,
                                   msg=lambda m: f"{n}: {m}")
    torch.testing.assert_close(model.bn1.running_mean, ref.bn1.running_mean, atol=1e-6,
                               rtol=1e-5)
    torch.testing.assert_close(model.bn1.running_var, ref.bn1.running_var, atol=1e-5, rtol=1e-5)
    tdp.destroy_process_group()


def training_loop(rank, out_dir):
    from tutorial_torch_distributed_data_parallel_amd.data import (DeviceLoader,
                                                                    DistributedSampler,
                                                                    SyntheticDataset)
    from tutorial_torch_distributed_data_parallel_amd.train import run_training_loop
    from tutorial_torch_distributed_data_parallel_amd.utils import set_seed_based_on_rank

    r, ws = _init()
    set_seed_based_on_rank(r, base_seed=5)
    train = SyntheticDataset(96, (20,), 4, seed=1)
    test = SyntheticDataset(40, (20,), 4, seed=2)
    ts = DistributedSampler(train, num_replicas=ws, rank=r, shuffle=True)
    vs = DistributedSampler(test, num_replicas=ws, rank=r, shuffle=True)
    tl = DeviceLoader(train, 8, sampler=ts)
    vl = DeviceLoader(test, 10, sampler=vs)
    model = tdp.DDP(ToyMLP(in_features=20, hidden=(32,), num_classes=4))
    opt = tdp.optim.Adam(model.parameters(), lr=1e-2)
    hist = run_training_loop(model, tl, ts, vl, tdp.nn.CrossEntropyLoss(), opt,
                             torch.device("cpu"), r, out_dir, num_epochs=6, checkpoint_epoch=5,
                             json_log=os.path.join(out_dir, "log.jsonl"), verbose=False)
    assert hist[-1]["train_loss"] < hist[0]["train_loss"]
    assert hist[0]["train_n"] == 96 and hist[0]["test_n"] == 40
    allp = _gather([p.detach().clone() for p in model.parameters()])
    for a, b in zip(allp[0], allp[-1]):
        assert torch.equal(a, b)
    if r == 0:
        torch.save({k: v for k, v in model.state_dict().items()},
                   os.path.join(out_dir, "final_rank0.pt"))
    tdp.destroy_process_group()


def fault_worker(rank, out_dir):
    from tutorial_torch_distributed_data_parallel_amd.utils import fault

    r, ws = _init()
    model = tdp.DDP(ToyMLP(in_features=8, hidden=(8,), num_classes=2))
    x = torch.randn(4, 8)
    y = torch.randint(0, 2, (4,))
    for step in range(50):
        fault.maybe_inject(r, step)
        tdp.ops.cross_entropy(model(x), y).backward()
        if r == 0 and step > 10:
            import time

            time.sleep(0.05)  # the survivor blocks in the next collective until torn down
    tdp.destroy_process_group()


def unused_params(rank, out_dir):
    r, ws = _init()

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = torch.nn.Linear(4, 4)
            self.b = torch.nn.Linear(4, 4)

        def forward(self, x):
            return self.a(x)

    ddp = tdp.DDP(M(), find_unused_parameters=True)
    ddp(torch.randn(2, 4)).sum().backward()
    gb = ddp.module.b.weight.grad  # torch semantics: an unused parameter keeps grad None
    assert gb is None or torch.count_nonzero(gb) == 0
    assert ddp.module.a.weight.grad is not None
    ddp2 = tdp.DDP(M(), find_unused_parameters=False)
    try:
        ddp2(torch.randn(2, 4)).sum().backward()
        raised = False
    except RuntimeError as e:
        raised = "find_unused_parameters" in str(e)
    assert raised
    tdp.destroy_process_group()


def accelerate_worker(rank, out_dir):
    from tutorial_torch_distributed_data_parallel_amd.accelerate import Accelerator
    from tutorial_torch_distributed_data_parallel_amd.data import DeviceLoader, SyntheticDataset

    acc = Accelerator(cpu=True)
    assert acc.num_processes == 2 and acc.process_index == rank
    ds = SyntheticDataset(40, (6,), 3, seed=0)
    loader = DeviceLoader(ds, 4)
    model = ToyMLP(in_features=6, hidden=(8,), num_classes=3)
    opt = torch.optim.Adam(model.parameters(), lr=1e-2)
    model, opt, loader = acc.prepare(model, opt, loader)
    seen = []
    for x, y in loader:
        seen.append(x)
        opt.zero_grad()
        loss = tdp.ops.cross_entropy(model(x), y)
        acc.backward(loss)
        opt.step()
    n = len(seen)
    counts = _gather(n)
    assert counts[0] == counts[1] == 5
    acc.wait_for_everyone()
    path = acc.save_model(model, out_dir)
    acc.wait_for_everyone()
    if acc.is_main_process:
        from safetensors.torch import load_file

        sd = load_file(path)
        assert all(not k.startswith("module.") for k in sd)
        assert set(sd) == set(acc.unwrap_model(model).state_dict())
    acc.end_training()


def replica_check(rank, out_dir):
    """SURVEY.md §5.2 debug mode: the replica checksum passes on healthy steps and names the
    diverged rank after one rank's parameters are corrupted."""
    import tutorial_torch_distributed_data_parallel_amd as tdp

    _init()
    torch.manual_seed(rank)
    model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))
    ddp = tdp.DDP(model, check_replicas_every=1)
    opt = tdp.optim.SGD(ddp.parameters(), lr=0.1)
    for _ in range(3):
        opt.zero_grad()
        ddp(torch.randn(5, 8)).sum().backward()
        opt.step()
    ddp.check_replicas()
    if rank == 1:
        with torch.no_grad():
            model[0].weight[0, 0] += 1e-3
    try:
        ddp(torch.randn(5, 8))
    except RuntimeError as e:
        assert "ranks [1]" in str(e), str(e)
    else:
        raise AssertionError("replica divergence not detected")
    tdp.destroy_process_group()
