"""Single-GPU end-to-end: RCCL communicator init, DDP over the native reducer, optimizers, and
parity of a full training step with stock torch (DDP semantics at world_size 1 = local grads)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg():
    import tutorial_torch_distributed_data_parallel_amd as tdp

    if not tdp.parallel.is_initialized():
        tdp.init_process_group("nccl", rank=0, world_size=1, local_rank=0)
    yield tdp
    tdp.destroy_process_group()


def test_rccl_collectives_ws1(pg):
    from tutorial_torch_distributed_data_parallel_amd.parallel import runtime as rt

    comm = rt.comm()
    assert comm is not None and comm.world == 1
    t = torch.arange(10, device="cuda", dtype=torch.float32)
    comm.all_reduce(t, "sum")
    comm.broadcast(t, 0)
    out = torch.empty(10, device="cuda")
    comm.all_gather(out, t)
    torch.testing.assert_close(out, torch.arange(10, device="cuda", dtype=torch.float32))
    rt.barrier()


@pytest.mark.parametrize("opt_name", ["sgd", "adam"])
@pytest.mark.parametrize("bn", [False, True])
def test_ddp_step_matches_torch(pg, opt_name, bn):
    tdp = pg
    from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP

    torch.manual_seed(0)
    model = ToyMLP(in_features=512, hidden=(256, 256), num_classes=10, batchnorm=bn,
                   device="cuda")
    ref = ToyMLP(in_features=512, hidden=(256, 256), num_classes=10, batchnorm=bn,
                 device="cuda")
    ref.load_state_dict(model.state_dict())
    ddp = tdp.DDP(model, device_ids=[0], bucket_cap_mb=0.25)
    if opt_name == "sgd":
        opt = tdp.optim.SGD(ddp.parameters(), lr=0.05, momentum=0.9)
        ropt = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9)
    else:
        opt = tdp.optim.Adam(ddp.parameters(), lr=1e-3)
        ropt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    x = torch.randn(64, 512, device="cuda")
    y = torch.randint(0, 10, (64,), device="cuda")
    for _ in range(3):
        opt.zero_grad(set_to_none=True)
        loss = tdp.ops.cross_entropy(ddp(x), y)
        loss.backward()
        opt.step()
        ropt.zero_grad(set_to_none=True)
        h = x
        for name in ref._order:
            mod = getattr(ref, name)
            if isinstance(mod, torch.nn.Linear):
                h = torch.nn.functional.linear(h, mod.weight, mod.bias)
                if getattr(mod, "relu", False):
                    h = torch.relu(h)
            else:
                h = torch.relu(torch.nn.functional.batch_norm(
                    h, mod.running_mean, mod.running_var, mod.weight, mod.bias, True, 0.1,
                    mod.eps))
        rloss = torch.nn.functional.cross_entropy(h, y)
        rloss.backward()
        ropt.step()
        torch.testing.assert_close(loss, rloss, atol=1e-4, rtol=1e-4)
    # gradients live in the arena (zero-copy buckets)
    for i, p in enumerate(ddp.arena.params):
        assert ddp.arena.is_arena_grad(i)
    # A Linear bias feeding a BatchNorm has an exactly-zero true gradient, so its computed
    # gradient is pure summation-order noise; Adam normalises that noise to +-lr per step.
    atol = 3.5e-3 if (bn and opt_name == "adam") else 2e-4
    for p, r in zip(model.parameters(), ref.parameters()):
        torch.testing.assert_close(p, r, atol=atol, rtol=1e-3)


def test_no_sync_accumulates(pg):
    tdp = pg
    from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP

    torch.manual_seed(1)
    model = ToyMLP(in_features=64, hidden=(32,), num_classes=10, device="cuda")
    ddp = tdp.DDP(model, device_ids=[0])
    x = torch.randn(16, 64, device="cuda")
    y = torch.randint(0, 10, (16,), device="cuda")
    with ddp.no_sync():
        tdp.ops.cross_entropy(ddp(x), y).backward()
    g1 = [p.grad.clone() for p in model.parameters()]
    tdp.ops.cross_entropy(ddp(x), y).backward()
    for p, g in zip(model.parameters(), g1):
        torch.testing.assert_close(p.grad, 2 * g, atol=1e-5, rtol=1e-5)


def test_captured_step_matches_eager(pg):
    """A hipGraph-replayed DDP step (train/graph.py) produces the eager step's results."""
    tdp = pg
    from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP
    from tutorial_torch_distributed_data_parallel_amd.train.graph import CapturedStep

    def build():
        torch.manual_seed(3)
        m = ToyMLP(in_features=256, hidden=(128, 128), num_classes=10, device="cuda")
        d = tdp.DDP(m, device_ids=[0])
        return m, d, tdp.optim.SGD(d.parameters(), lr=0.05, momentum=0.9)

    X = torch.randn(512, 256, device="cuda")
    Y = torch.randint(0, 10, (512,), device="cuda")
    idx = torch.zeros(64, dtype=torch.long, device="cuda")

    def make_step(d, opt):
        def step():
            x, y = X.index_select(0, idx), Y.index_select(0, idx)
            opt.zero_grad(set_to_none=True)
            loss = tdp.ops.cross_entropy(d(x), y)
            loss.backward()
            opt.step()
            return loss
        return step

    m1, d1, o1 = build()
    m2, d2, o2 = build()
    eager = make_step(d1, o1)
    orders = [torch.randperm(512, device="cuda")[:64] for _ in range(8)]
    # CapturedStep runs 3 real warm-up steps; the capture itself records without executing
    idx.copy_(orders[0])
    for _ in range(3):
        eager()
    graph = CapturedStep(make_step(d2, o2), warmup=3)
    for o in orders[1:]:
        idx.copy_(o)
        le = eager()
        lg = graph.replay()
        torch.testing.assert_close(lg, le, atol=1e-5, rtol=1e-5)
    for a, b in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-4)


def test_captured_step_keeps_ddp_host_bookkeeping(pg):
    """Replays advance DDP's iteration counter like eager steps (the capture itself does not
    count), check_replicas_every fires after replays, and find_unused_parameters=True refuses
    capture (the per-iteration unused set is host logic) so try_capture runs eagerly."""
    tdp = pg
    from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP
    from tutorial_torch_distributed_data_parallel_amd.train import graph as G

    torch.manual_seed(5)
    m = ToyMLP(in_features=128, hidden=(64,), num_classes=10, device="cuda")
    d = tdp.DDP(m, device_ids=[0], check_replicas_every=2)
    o = tdp.optim.SGD(d.parameters(), lr=0.05, momentum=0.9)
    x = torch.randn(32, 128, device="cuda")
    y = torch.randint(0, 10, (32,), device="cuda")
    calls = []
    d.check_replicas = lambda: calls.append(d._iter)

    def step():
        o.zero_grad(set_to_none=True)
        tdp.ops.backward(tdp.ops.cross_entropy(d(x), y))
        o.step()

    g = G.CapturedStep(step, warmup=3)
    assert d._iter == 3  # three real warm-up steps; recording the graph is not a step
    calls.clear()
    for _ in range(5):
        g.replay()
    assert d._iter == 8
    assert calls == [4, 6, 8]
    del g

    m2 = ToyMLP(in_features=128, hidden=(64,), num_classes=10, device="cuda")
    d2 = tdp.DDP(m2, device_ids=[0], find_unused_parameters=True)
    o2 = tdp.optim.SGD(d2.parameters(), lr=0.05)

    def step2():
        o2.zero_grad(set_to_none=True)
        tdp.ops.backward(tdp.ops.cross_entropy(d2(x), y))
        o2.step()

    logs = []
    got = G.try_capture(step2, warmup=1, log=logs.append)
    assert got is step2 and "find_unused_parameters" in logs[0]
    it = d2._iter
    got()
    assert d2._iter == it + 1
    del d2, d


@pytest.mark.parametrize("opt_name", ["sgd", "adam"])
def test_fused_optimizer_matches_unfused(pg, opt_name):
    """Optimizer applied per bucket inside the reduction == optimizer.step() after backward."""
    tdp = pg
    from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP

    def build(fused):
        torch.manual_seed(4)
        m = ToyMLP(in_features=256, hidden=(192, 128), num_classes=10, device="cuda")
        d = tdp.DDP(m, device_ids=[0], bucket_cap_mb=0.05, first_bucket_cap_mb=0.004)
        o = (tdp.optim.SGD(d.parameters(), lr=0.05, momentum=0.9) if opt_name == "sgd"
             else tdp.optim.Adam(d.parameters(), lr=1e-3))
        if fused:
            assert d.register_fused_optimizer(o)
        return m, d, o

    m1, d1, o1 = build(False)
    m2, d2, o2 = build(True)
    assert d2._get_ddp_logging_data()["num_buckets"] >= 3
    for i in range(4):
        x = torch.randn(64, 256, device="cuda")
        y = torch.randint(0, 10, (64,), device="cuda")
        for d, o in ((d1, o1), (d2, o2)):
            o.zero_grad(set_to_none=True)
            tdp.ops.cross_entropy(d(x), y).backward()
            o.step()
        if i == 1:  # LR change reaches the fused path through step()
            for o in (o1, o2):
                o.param_groups[0]["lr"] *= 0.5
    torch.cuda.synchronize()
    for a, b in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a, b, atol=1e-6, rtol=1e-5)
    sd = o2.state_dict()
    assert len(sd["state"]) == len(list(m2.parameters()))


@pytest.mark.parametrize("bn", [False, True])
@pytest.mark.parametrize("opt_name", ["sgd", "adam", "sgd_nesterov_wd"])
def test_optimizer_epilogue_matches_bucket_update(pg, opt_name, bn, monkeypatch):
    """World size 1: the optimizer applied in the weight-gradient GEMM epilogue (gradient never
    stored) == the per-bucket fused update == optimizer.step() after backward; with BatchNorm1d
    layers (bn) their affine parameters are updated inside the one-launch BN backward."""
    tdp = pg
    from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP

    def build(mode):
        monkeypatch.setenv("TDP_OPT_EPILOGUE", "1" if mode == "epilogue" else "0")
        torch.manual_seed(5)
        m = ToyMLP(in_features=512, hidden=(384, 256), num_classes=10, batchnorm=bn,
                   device="cuda")
        d = tdp.DDP(m, device_ids=[0], bucket_cap_mb=0.5, first_bucket_cap_mb=0.02)
        if opt_name == "sgd":
            o = tdp.optim.SGD(d.parameters(), lr=0.05, momentum=0.9)
        elif opt_name == "sgd_nesterov_wd":
            o = tdp.optim.SGD(d.parameters(), lr=0.05, momentum=0.9, nesterov=True,
                              weight_decay=1e-3)
        else:
            o = tdp.optim.Adam(d.parameters(), lr=1e-3)
        if mode != "plain":
            assert d.register_fused_optimizer(o)
        assert d._epi_on == (mode == "epilogue")
        return m, d, o

    runs = [build(mode) for mode in ("plain", "bucket", "epilogue")]
    for i in range(4):
        x = torch.randn(128, 512, device="cuda")
        y = torch.randint(0, 10, (128,), device="cuda")
        for m, d, o in runs:
            o.zero_grad(set_to_none=True)
            tdp.ops.cross_entropy(d(x), y).backward()
            o.step()
        if i == 1:
            for _, _, o in runs:
                o.param_groups[0]["lr"] *= 0.5
    torch.cuda.synchronize()
    ref = dict(runs[0][0].named_parameters())
    # a Linear bias feeding a BatchNorm has an exactly-zero true gradient: its computed gradient
    # is summation-order noise, which Adam normalises to +-lr per step (test_ddp_step_matches_torch)
    noise = {"fc1.bias", "fc2.bias"} if (bn and opt_name == "adam") else set()
    for m, _, _ in runs[1:]:
        for name, b in m.named_parameters():
            atol = 3.5e-3 if name in noise else 2e-6
            torch.testing.assert_close(b, ref[name], atol=atol, rtol=1e-5, msg=name)
    if bn:
        # the BN affine parameters were updated by the BN backward kernel, not the bucket pass
        d = runs[2][1]
        bn_mods = [mod for mod in runs[2][0].modules()
                   if isinstance(mod, torch.nn.modules.batchnorm._BatchNorm)]
        assert bn_mods and d._epi_on


def test_capture_right_after_first_step_with_pending_rebuild(pg):
    """a bucket rebuild planned by iteration 0 must not be recorded into the graph
    (every replay would restore the pre-capture buffers). CapturedStep(warmup=1) settles it
    eagerly first: replays must keep changing the parameters, exactly like eager steps."""
    tdp = pg
    from tutorial_torch_distributed_data_parallel_amd.train.graph import CapturedStep

    class Shuffled(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = tdp.nn.Linear(64, 128, relu=True)
            self.c = tdp.nn.Linear(128, 10)          # registered second, runs last
            self.b = tdp.nn.Linear(128, 128, relu=True)

        def forward(self, x):
            return self.c(self.b(self.a(x)))

    def build():
        torch.manual_seed(5)
        m = Shuffled().cuda()
        d = tdp.DDP(m, device_ids=[0], bucket_cap_mb=100 / 2 ** 20,
                    first_bucket_cap_mb=100 / 2 ** 20)
        return m, d, tdp.optim.SGD(d.parameters(), lr=0.05, momentum=0.9)

    x = torch.randn(32, 64, device="cuda")
    y = torch.randint(0, 10, (32,), device="cuda")

    def make(d, o):
        def step():
            o.zero_grad(set_to_none=True)
            loss = tdp.ops.cross_entropy(d(x), y)
            loss.backward()
            o.step()
            return loss
        return step

    m1, d1, o1 = build()
    m2, d2, o2 = build()
    eager = make(d1, o1)
    eager()
    graph = CapturedStep(make(d2, o2), warmup=1)
    assert d2._rebuilt, "the warm-up step should have planned a rebuild, settled before capture"
    before = [p.detach().clone() for p in m2.parameters()]
    for _ in range(3):
        eager()
        graph.replay()
    torch.cuda.synchronize()
    assert any(not torch.equal(a, b) for a, b in zip(before, m2.parameters()))
    for a, b in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-4)
