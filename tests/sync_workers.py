"""Multi-rank workers for the gradient-sync algorithm (csrc/reducer.cpp SyncBackend) on CPU/gloo.

The C++ SyncBackend drives parallel/ddp.py ``_CpuSyncOps`` here exactly as it drives RcclOps on
MI355X, so these runs exercise the production bucket order, the sharded reduce-scatter -> 1/W
update -> all-gather path with tails that do not divide by W, in-reduction clipping, device-style
hyper blocks (LR changes, Adam step count) and state consolidation for checkpoints, at world
sizes 2 and 3. The oracle is stock ``torch.nn.parallel.DistributedDataParallel`` +
``torch.optim`` on the same data (SURVEY.md §4.3 oracles 1-2).
"""
import copy
import os

import torch
import torch.distributed as dist
import torch.nn.functional as F

import tutorial_torch_distributed_data_parallel_amd as tdp
from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP
from tutorial_torch_distributed_data_parallel_amd.parallel import runtime as rt

# odd layer sizes: no parameter, bucket or arena size divides evenly by 2 or 3
DIMS = dict(in_features=37, hidden=(29, 23), num_classes=5)
# ~1.9k parameters: 2 KiB buckets, params above 1.5 KiB split -> ~6 buckets with shard tails
BUCKETS = dict(bucket_cap_mb=2048 / 2 ** 20, first_bucket_cap_mb=600 / 2 ** 20,
               split_bucket_mb=1536 / 2 ** 20)


def _gather(obj):
    out = [None] * rt.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def _make_opts(kind, ours_params, ref_params, lr):
    if kind == "sgd":
        hp = dict(lr=lr, momentum=0.9, weight_decay=1e-3, nesterov=True)
        return tdp.optim.SGD(ours_params, **hp), torch.optim.SGD(ref_params, **hp)
    if kind == "adamw":
        hp = dict(lr=lr, weight_decay=5e-2)
        return tdp.optim.AdamW(ours_params, **hp), torch.optim.AdamW(ref_params, **hp)
    hp = dict(lr=lr, weight_decay=1e-3, amsgrad=kind == "amsgrad")
    return tdp.optim.Adam(ours_params, **hp), torch.optim.Adam(ref_params, **hp)


def _batch(r, step):
    g = torch.Generator().manual_seed(1000 * step + r)
    return torch.randn(6, 37, generator=g) * (1 + r), torch.randint(0, 5, (6,), generator=g)


def _check_close(model, ref, tag, atol=2e-5):
    for (n, p), (_, q) in zip(model.named_parameters(), ref.named_parameters()):
        torch.testing.assert_close(p.detach(), q.detach(), atol=atol, rtol=1e-4,
                                   msg=lambda m: f"{tag} {n}: {m}")


def _check_replicas(model):
    allp = _gather([p.detach().clone() for p in model.parameters()])
    for other in allp[1:]:
        for a, b in zip(other, allp[0]):
            assert torch.equal(a, b), "replicas diverged"


def _teardown():
    # stock torch DDP objects (dropped by the caller) must die before their process group does:
    # their reducer / gloo work threads otherwise abort the process at exit
    import gc

    gc.collect()
    dist.barrier()
    tdp.destroy_process_group()


def fused_parity(rank, out_dir, kind="sgd", shard=True, clip=None, steps=5):
    """Fused (in-reduction) optimizer vs torch DDP + torch.optim, with an LR change mid-run,
    then consolidate -> save -> load into fresh objects -> continue."""
    tdp.init_process_group("gloo")
    r = rt.get_rank()
    torch.manual_seed(0)
    model = ToyMLP(**DIMS)
    ref = copy.deepcopy(model)
    ddp = tdp.DDP(model, **BUCKETS)
    assert ddp._backend.collective
    opt, ropt = _make_opts(kind, ddp.parameters(), ref.parameters(), 0.05 if kind == "sgd"
                           else 1e-2)
    assert ddp.register_fused_optimizer(opt, shard=shard, clip_grad_norm=clip)
    nb = len(ddp._bounds) - 1
    assert nb >= 4, ddp._bounds
    rddp = torch.nn.parallel.DistributedDataParallel(ref)

    def both_steps(n0, n1):
        for step in range(n0, n1):
            if step == 3:  # LR schedule: the fused update must see the new value
                for o in (opt, ropt):
                    o.param_groups[0]["lr"] *= 0.5
            x, y = _batch(r, step)
            opt.zero_grad()
            tdp.ops.cross_entropy(ddp(x), y).backward()
            opt.step()  # no-op: the update ran inside the reduction
            ropt.zero_grad()
            F.cross_entropy(rddp(x), y).backward()
            if clip:
                torch.nn.utils.clip_grad_norm_(rddp.parameters(), clip)
            ropt.step()
        _check_close(model, ref, f"{kind} shard={shard} clip={clip} after {n1} steps")
        _check_replicas(model)

    both_steps(0, steps)
    if clip:
        norm = float(ddp.last_grad_norm())
        assert norm > 0
    # checkpoint: consolidate the sharded state, every rank holds the complete optimizer state
    ddp.consolidate_optimizer_state()
    sd = opt.state_dict()
    rsd = ropt.state_dict()
    for pid, st in rsd["state"].items():
        for k, v in st.items():
            if k == "step":
                assert int(sd["state"][pid]["step"]) == int(v), (k, sd["state"][pid]["step"], v)
            else:
                torch.testing.assert_close(sd["state"][pid][k], v, atol=2e-5, rtol=1e-4,
                                           msg=lambda m: f"state {pid}.{k}: {m}")
    path = os.path.join(out_dir, f"state_{r}.pt")
    torch.save({"model": {k: v.clone() for k, v in model.state_dict().items()}, "opt": sd}, path)
    dist.barrier()
    # fresh objects: load, register, continue; must track the reference exactly as before
    ck = torch.load(path, weights_only=True)
    torch.manual_seed(123)
    model2 = ToyMLP(**DIMS)
    model2.load_state_dict(ck["model"])
    ddp2 = tdp.DDP(model2, **BUCKETS)
    opt2, _ = _make_opts(kind, ddp2.parameters(), [torch.nn.Parameter(torch.zeros(1))], 1.0)
    opt2.load_state_dict(ck["opt"])
    ddp2.register_fused_optimizer(opt2, shard=shard, clip_grad_norm=clip)
    model, ddp, opt = model2, ddp2, opt2
    both_steps(steps, steps + 2)
    rddp = None  # noqa: F841
    _teardown()


def local_clip_parity(rank, out_dir, max_norm=0.05, fused=True):
    """README pitfall (REF/README.md:92-95): every rank clips its OWN gradient before the
    average. Oracle: per-rank torch clip_grad_norm_ on a plain model, manual average, step."""
    tdp.init_process_group("gloo")
    r, W = rt.get_rank(), rt.get_world_size()
    torch.manual_seed(0)
    model = ToyMLP(**DIMS)
    ref = copy.deepcopy(model)
    ddp = tdp.DDP(model, **BUCKETS)
    ddp.clip_grad_norm_before_aggregation(max_norm)
    opt = tdp.optim.SGD(ddp.parameters(), lr=0.1, momentum=0.9)
    ropt = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=0.9)
    if fused:
        ddp.register_fused_optimizer(opt)
    for step in range(4):
        x, y = _batch(r, step)
        opt.zero_grad()
        tdp.ops.cross_entropy(ddp(x), y).backward()
        opt.step()
        ropt.zero_grad()
        F.cross_entropy(ref(x), y).backward()
        n = torch.nn.utils.clip_grad_norm_(ref.parameters(), max_norm)
        assert float(n) > max_norm  # the clip is active
        for p in ref.parameters():
            dist.all_reduce(p.grad)
            p.grad.div_(W)
        ropt.step()
        torch.testing.assert_close(ddp.last_grad_norm(), n, atol=1e-5, rtol=1e-4)
    _check_close(model, ref, f"local clip fused={fused}")
    _check_replicas(model)
    tdp.destroy_process_group()


def comm_hook_keeps_fused_state(rank, out_dir):
    """register_comm_hook after register_fused_optimizer must keep the Adam step count,
    the shard flag and the state buffers."""
    tdp.init_process_group("gloo")
    r = rt.get_rank()
    torch.manual_seed(0)
    model = ToyMLP(**DIMS)
    ref = copy.deepcopy(model)
    ddp = tdp.DDP(model, **BUCKETS)
    opt, ropt = _make_opts("adam", ddp.parameters(), ref.parameters(), 1e-2)
    ddp.register_fused_optimizer(opt)
    rddp = torch.nn.parallel.DistributedDataParallel(ref)
    for step in range(4):
        if step == 2:
            ddp.register_comm_hook(None, "fp32")  # rebuilds the reducer backend
            assert ddp._backend.shard and ddp._backend.fused_kind == 2
        x, y = _batch(r, step)
        opt.zero_grad()
        tdp.ops.cross_entropy(ddp(x), y).backward()
        ropt.zero_grad()
        F.cross_entropy(rddp(x), y).backward()
        ropt.step()
    assert opt.device_step(0) == 4
    _check_close(model, ref, "comm hook rebuild")
    rddp = None  # noqa: F841
    _teardown()


def shared_parameter(rank, out_dir):
    """one Linear applied twice in a forward. The gradient is the SUM of both
    uses' contributions, averaged over ranks."""
    tdp.init_process_group("gloo")
    r = rt.get_rank()

    class Twice(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.inp = tdp.nn.Linear(10, 16, relu=True)
            self.mid = tdp.nn.Linear(16, 16, relu=True)  # applied twice
            self.out = tdp.nn.Linear(16, 4)

        def forward(self, x):
            return self.out(self.mid(self.mid(self.inp(x))))

    torch.manual_seed(0)
    model = Twice()
    ref = copy.deepcopy(model)
    ddp = tdp.DDP(model)
    rddp = torch.nn.parallel.DistributedDataParallel(ref)
    g = torch.Generator().manual_seed(r)
    x, y = torch.randn(8, 10, generator=g), torch.randint(0, 4, (8,), generator=g)
    tdp.ops.cross_entropy(ddp(x), y).backward()
    F.cross_entropy(rddp(x), y).backward()
    for (n, p), (_, q) in zip(model.named_parameters(), ref.named_parameters()):
        torch.testing.assert_close(p.grad, q.grad, atol=1e-6, rtol=1e-5,
                                   msg=lambda m: f"{n}: {m}")
    rddp = None  # noqa: F841
    _teardown()


def logger_stats(rank, out_dir):
    """DDP Logger: sampled forward / backward / comm times and bucket info."""
    tdp.init_process_group("gloo")
    torch.manual_seed(0)
    ddp = tdp.DDP(ToyMLP(**DIMS), timing=True, **BUCKETS)
    for step in range(3):
        x, y = _batch(rt.get_rank(), step)
        tdp.ops.cross_entropy(ddp(x), y).backward()
    info = ddp._get_ddp_logging_data()
    assert info["sampled_iterations"] == 3, info
    assert info["avg_forward_compute_time_ms"] > 0 and info["avg_backward_compute_time_ms"] > 0
    assert info["avg_backward_exposed_comm_time_ms"] >= 0
    assert info["num_buckets"] == len(info["bucket_sizes"]) >= 4
    assert info["head_of_line_waits"] == 0  # a sequential model: buckets become ready in order
    tdp.destroy_process_group()


def bucket_rebuild(rank, out_dir, fused=True):
    """Bucket rebuild (torch DDP ``_rebuild_buckets``): layers registered in a different order
    than they run, one bucket per parameter -> head-of-line waits in iteration 0 -> the arena is
    re-laid out in ready order, and training (sharded fused Adam at W=2) still matches torch."""
    tdp.init_process_group("gloo")
    r = rt.get_rank()

    class Shuffled(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = tdp.nn.Linear(12, 40, relu=True)
            self.c = tdp.nn.Linear(40, 5)          # registered second, runs last
            self.b = tdp.nn.Linear(40, 40, relu=True)

        def forward(self, x):
            return self.c(self.b(self.a(x)))

    torch.manual_seed(0)
    model = Shuffled()
    ref = copy.deepcopy(model)
    ddp = tdp.DDP(model, bucket_cap_mb=100 / 2 ** 20, first_bucket_cap_mb=100 / 2 ** 20)
    opt = tdp.optim.Adam(ddp.parameters(), lr=1e-2)
    ropt = torch.optim.Adam(ref.parameters(), lr=1e-2)
    if fused:
        ddp.register_fused_optimizer(opt)
    rddp = torch.nn.parallel.DistributedDataParallel(ref)
    for step in range(5):
        g = torch.Generator().manual_seed(100 * step + r)
        x, y = torch.randn(8, 12, generator=g), torch.randint(0, 5, (8,), generator=g)
        opt.zero_grad()
        tdp.ops.cross_entropy(ddp(x), y).backward()
        opt.step()
        ropt.zero_grad()
        F.cross_entropy(rddp(x), y).backward()
        ropt.step()
        if step == 0:
            assert ddp.reducer.head_of_line_waits > 0
            assert ddp._rebuild_order is not None
        if step == 1:
            assert ddp._rebuilt and ddp.reducer.head_of_line_waits == 0
    assert ddp._get_ddp_logging_data()["has_rebuilt_buckets"] == 1
    _check_close(model, ref, f"after rebuild fused={fused}")
    _check_replicas(model)
    rddp = None  # noqa: F841
    _teardown()


# factored Linear synchronisation (csrc/reducer.h FactorJob) on the gloo twin: fc1 [96, 96] and
# fc2 [48, 96] are factored at W = 2..4 (out % 4W == 0, whole-row 64-element shards, and
# 2 W B (out + in) <= out * in at B = 4); the 5-class head stays on the bucket path
FACTOR_DIMS = dict(in_features=96, hidden=(96, 48), num_classes=5)


def _factor_batch(r, step, W, ragged_step):
    g = torch.Generator().manual_seed(1000 * step + r)
    # a ragged last batch on the last rank (DataLoader drop_last=False): fewer rows than agreed
    b = 2 if (step == ragged_step and r == W - 1) else 4
    return torch.randn(b, 96, generator=g) * (1 + r), torch.randint(0, 5, (b,), generator=g)


def factored_parity(rank, out_dir, kind="sgd", replicate=False, steps=5):
    """Factored sync (all-gather of g / W and x, depth-W*B row-shard GEMM, bias from the column
    sums, sharded or replicated update) vs stock torch DDP + torch.optim: LR change at step 3,
    a ragged batch on one rank at step 4 (zero-padded into the agreed slot), unowned gradient
    rows poisoned with NaN, replicas bit-identical."""
    tdp.init_process_group("gloo")
    r, W = rt.get_rank(), rt.get_world_size()
    torch.manual_seed(0)
    model = ToyMLP(**FACTOR_DIMS)
    ref = copy.deepcopy(model)
    ddp = tdp.DDP(model, factor_sync=True)
    if replicate == "mixed":  # per weight, by parameter name (survives the bucket rebuild)
        replicate = {"fc1.weight": True, "fc2.weight": False}
    ddp.factor_replicate = replicate
    opt, ropt = _make_opts(kind, ddp.parameters(), ref.parameters(), 0.05 if kind == "sgd"
                           else 1e-2)
    assert ddp.register_fused_optimizer(opt)
    assert len(ddp._factor) == 2, ddp._factor
    rddp = torch.nn.parallel.DistributedDataParallel(ref)
    for step in range(steps):
        if step == 3:
            for o in (opt, ropt):
                o.param_groups[0]["lr"] *= 0.5
        x, y = _factor_batch(r, step, W, ragged_step=4)
        opt.zero_grad()
        tdp.ops.cross_entropy(ddp(x), y).backward()
        opt.step()
        ropt.zero_grad()
        F.cross_entropy(rddp(x), y).backward()
        ropt.step()
        plan = ddp.sync_plan()
        for n in ("fc1.weight", "fc2.weight"):
            rep = replicate.get(n) if isinstance(replicate, dict) else replicate
            want = "factored-replicated" if rep else "factored-sharded"
            assert plan[n] == want, (n, plan)
        assert plan["fc1.bias"] == "factored-bias" and plan["fc3.weight"] == "sharded", plan
    assert set(ddp._factor_cap.values()) == {4}, ddp._factor_cap
    _check_close(model, ref, f"factored {kind} replicate={replicate} W={W}", atol=3e-5)
    _check_replicas(model)
    ddp.check_replicas()
    # consolidated optimizer state equals torch's (the sharded state slices are gathered)
    ddp.consolidate_optimizer_state()
    sd, rsd = opt.state_dict(), ropt.state_dict()
    for pid, st in rsd["state"].items():
        for k, v in st.items():
            if k != "step":
                torch.testing.assert_close(sd["state"][pid][k], v, atol=3e-5, rtol=1e-4,
                                           msg=lambda m: f"state {pid}.{k}: {m}")
    rddp = None  # noqa: F841
    _teardown()


def factored_foreign_gradient(rank, out_dir):
    """another op adding to a factored weight's gradient (an L2 penalty) must raise,
    not be silently dropped by the factored job."""
    import pytest

    tdp.init_process_group("gloo")
    torch.manual_seed(0)
    model = ToyMLP(**FACTOR_DIMS)
    ddp = tdp.DDP(model, factor_sync=True)
    opt = tdp.optim.SGD(ddp.parameters(), lr=0.05, momentum=0.9)
    ddp.register_fused_optimizer(opt)
    x, y = _factor_batch(rt.get_rank(), 0, rt.get_world_size(), ragged_step=-1)
    loss = tdp.ops.cross_entropy(ddp(x), y) + 1e-3 * (model.fc1.weight ** 2).sum()
    with pytest.raises(RuntimeError, match="factored"):
        loss.backward()
    dist.barrier()
    tdp.destroy_process_group()


def capture_agreement(rank, out_dir):
    """A capture failure on ONE rank makes every rank run eagerly (train/graph.py try_capture)."""
    from tutorial_torch_distributed_data_parallel_amd.train import graph as G

    tdp.init_process_group("gloo")
    r = rt.get_rank()

    class FakeCapture:
        def __init__(self, fn, warmup=3):
            if r == 1:
                raise G.CaptureFailed("injected on rank 1")
            self.fn = fn

    def step():
        return None

    got = G.try_capture(step, warmup=1, log=lambda m: None, capture=FakeCapture)
    assert got is step, f"rank {r} kept a captured step while rank 1 runs eagerly"
    # and with no failure anywhere every rank keeps its graph
    ok = G.try_capture(step, warmup=1, log=lambda m: None,
                       capture=lambda fn, warmup=3: ("graph", fn))
    assert ok != step
    tdp.destroy_process_group()


def accumulation_parity(rank, out_dir, fused=False, gas=4, steps=8):
    """Accelerator.accumulate (ACC/accelerator.py accumulate / no_sync): non-synchronising
    micro-steps issue no collective and accumulate locally; every gas-th one averages and
    steps. Oracle: torch DDP with no_sync and a manual 1/gas loss scale."""
    import contextlib

    from tutorial_torch_distributed_data_parallel_amd.accelerate import Accelerator

    tdp.init_process_group("gloo")
    r = rt.get_rank()
    torch.manual_seed(0)
    model = ToyMLP(**DIMS)
    ref = copy.deepcopy(model)
    acc = Accelerator(gradient_accumulation_steps=gas)
    model, opt = acc.prepare(model, tdp.optim.SGD(model.parameters(), lr=0.05, momentum=0.9))
    if fused:
        assert model.register_fused_optimizer(opt.optimizer)
    rddp = torch.nn.parallel.DistributedDataParallel(ref)
    ropt = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9)
    for i in range(steps):
        x, y = _batch(r, i)
        with acc.accumulate(model):
            acc.backward(tdp.ops.cross_entropy(model(x), y))
            opt.step()
            opt.zero_grad()
        sync = (i + 1) % gas == 0
        assert acc.sync_gradients == sync
        with (contextlib.nullcontext() if sync else rddp.no_sync()):
            (F.cross_entropy(rddp(x), y) / gas).backward()
        if sync:
            ropt.step()
            ropt.zero_grad()
    # one reducer iteration (bucket collectives) per synchronising micro-step only
    assert model._get_ddp_logging_data()["iterations"] == steps // gas
    _check_close(model, ref, f"accumulate gas={gas} fused={fused}")
    _check_replicas(model)
    rddp = None  # noqa: F841
    _teardown()


def rebuild_moves_shards(rank, out_dir, kind="sgd"):
    """A bucket rebuild under the SHARDED fused optimizer moves parameters across shard owners
    (layers registered in a different order than they run, several parameters per bucket):
    optimizer state that was current only on the old owner must reach the new one (the rebuild
    consolidates it first). Oracle: torch DDP + torch.optim."""
    tdp.init_process_group("gloo")
    r = rt.get_rank()

    class Shuffled(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = tdp.nn.Linear(24, 40, relu=True)
            self.c = tdp.nn.Linear(40, 6)           # registered second, runs last
            self.b = tdp.nn.Linear(40, 40, relu=True)

        def forward(self, x):
            return self.c(self.b(self.a(x)))

    torch.manual_seed(0)
    model = Shuffled()
    ref = copy.deepcopy(model)
    ddp = tdp.DDP(model, bucket_cap_mb=250 * 4 / 2 ** 20, first_bucket_cap_mb=200 * 4 / 2 ** 20)
    opt, ropt = _make_opts(kind, ddp.parameters(), ref.parameters(), 0.05 if kind == "sgd"
                           else 1e-2)
    ddp.register_fused_optimizer(opt)
    rddp = torch.nn.parallel.DistributedDataParallel(ref)
    for step in range(5):
        g = torch.Generator().manual_seed(100 * step + r)
        x, y = torch.randn(8, 24, generator=g), torch.randint(0, 6, (8,), generator=g)
        opt.zero_grad()
        tdp.ops.cross_entropy(ddp(x), y).backward()
        ropt.zero_grad()
        F.cross_entropy(rddp(x), y).backward()
        ropt.step()
        if step == 0:
            assert ddp._rebuild_order is not None, "expected a rebuild"
    assert ddp._rebuilt
    _check_close(model, ref, f"rebuild moves shards {kind}")
    _check_replicas(model)
    rddp = None  # noqa: F841
    _teardown()


def factored_tuning(rank, out_dir, steps_after=2):
    """DDP.tune_factor_replicate on the CPU twin: every replicated / sharded combination of the
    two factored weights timed on real training steps (max over ranks), the choice recorded
    by parameter NAME and applied (it survives the bucket rebuild the first step triggers);
    every tuning step is a real step, so the model still matches torch DDP run over the same
    batches, and the replicas stay identical."""
    tdp.init_process_group("gloo")
    r, W = rt.get_rank(), rt.get_world_size()
    torch.manual_seed(0)
    model = ToyMLP(**FACTOR_DIMS)
    ref = copy.deepcopy(model)
    ddp = tdp.DDP(model, factor_sync=True)
    opt, ropt = _make_opts("sgd", ddp.parameters(), ref.parameters(), 0.05)
    assert ddp.register_fused_optimizer(opt)
    rddp = torch.nn.parallel.DistributedDataParallel(ref)
    k = [0]

    def step():
        x, y = _factor_batch(r, k[0], W, ragged_step=-1)
        k[0] += 1
        opt.zero_grad()
        tdp.ops.cross_entropy(ddp(x), y).backward()
        opt.step()

    got = ddp.tune_factor_replicate(step, iters=1)
    tun = ddp.factor_tuning
    assert set(got) == {"fc1.weight", "fc2.weight"}, got
    assert set(tun["chosen"]) == {"fc1.weight", "fc2.weight"}, tun
    assert len(tun["timings_ms"]) == 4 and tun["captured"] is False, tun
    for _ in range(steps_after):
        step()
    plan = ddp.sync_plan()
    for n, c in tun["chosen"].items():
        assert plan[n] == "factored-" + c, (n, c, plan)
    for i in range(k[0]):
        x, y = _factor_batch(r, i, W, ragged_step=-1)
        ropt.zero_grad()
        F.cross_entropy(rddp(x), y).backward()
        ropt.step()
    _check_close(model, ref, "factored after tuning", atol=3e-5)
    ddp.check_replicas()
    rddp = None  # noqa: F841
    _teardown()


def factored_batch_over_slot(rank, out_dir, agree_first=False):
    """a per-rank batch above the agreed factor slot on ONE rank only.
    Without factor_capacity the over-slot rank raises cleanly (no collective from a subset of
    the ranks, which would pair with the others' factor all-gathers and hang); the launcher's
    fail-fast ends the job. With factor_capacity(6) agreed up front every rank runs the step
    and matches stock torch DDP."""
    tdp.init_process_group("gloo")
    r, W = rt.get_rank(), rt.get_world_size()
    torch.manual_seed(0)
    model = ToyMLP(**FACTOR_DIMS)
    ref = copy.deepcopy(model)
    ddp = tdp.DDP(model, factor_sync=True)
    opt, ropt = _make_opts("sgd", ddp.parameters(), ref.parameters(), 0.05)
    ddp.register_fused_optimizer(opt)
    if agree_first:
        ddp.factor_capacity(6 if r == 0 else 4)  # the max over ranks is agreed
    rddp = torch.nn.parallel.DistributedDataParallel(ref)
    for step in range(3):
        x, y = _factor_batch(r, step, W, ragged_step=-1)
        if step == 1 and r == 0:  # one rank's batch grows past the first step's slot
            g = torch.Generator().manual_seed(77)
            x, y = torch.randn(6, 96, generator=g), torch.randint(0, 5, (6,), generator=g)
        opt.zero_grad()
        tdp.ops.cross_entropy(ddp(x), y).backward()
        opt.step()
        ropt.zero_grad()
        F.cross_entropy(rddp(x), y).backward()
        ropt.step()
    assert set(ddp._factor_cap.values()) == {6}, ddp._factor_cap
    _check_close(model, ref, "factored over-slot batch", atol=3e-5)
    _check_replicas(model)
    rddp = None  # noqa: F841
    _teardown()
