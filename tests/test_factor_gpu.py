"""Factored gradient synchronisation of Linear weights (reducer.h FactorJob, DDP._factor_candidates)
on one GPU: the single-GPU rehearsal (collectives forced at world size 1) runs the real device
path -- factor staging, RCCL all-gathers, the depth-W*B shard GEMM with the fused optimizer in its
epilogue, the parameter all-gather -- and must train exactly like the ordinary bucket path and
like torch.optim over F.linear."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg():
    import tutorial_torch_distributed_data_parallel_amd as tdp

    if not tdp.parallel.is_initialized():
        tdp.init_process_group("nccl", rank=0, world_size=1, local_rank=0)
    yield tdp
    tdp.destroy_process_group()


DIMS = (512, (256, 128))


def _build(tdp, opt_name, factor, seed=11):
    from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP

    torch.manual_seed(seed)
    m = ToyMLP(in_features=DIMS[0], hidden=DIMS[1], num_classes=10, device="cuda")
    d = tdp.DDP(m, device_ids=[0], force_collective=True, factor_sync=factor)
    o = (tdp.optim.SGD(d.parameters(), lr=0.05, momentum=0.9) if opt_name == "sgd"
         else tdp.optim.Adam(d.parameters(), lr=1e-3))
    assert d.register_fused_optimizer(o)
    return m, d, o


def _torch_step(ref, ropt, x, y):
    ropt.zero_grad(set_to_none=True)
    h = x
    for name in ref._order:
        mod = getattr(ref, name)
        h = F.linear(h, mod.weight, mod.bias)
        if getattr(mod, "relu", False):
            h = torch.relu(h)
    loss = F.cross_entropy(h, y)
    loss.backward()
    ropt.step()
    return loss


@pytest.mark.parametrize("opt_name", ["sgd", "adam"])
def test_factored_matches_bucket_path_and_torch(pg, opt_name):
    tdp = pg
    from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP

    m1, d1, o1 = _build(tdp, opt_name, True)
    m2, d2, o2 = _build(tdp, opt_name, False)
    # fc1 (256 x 512) and fc2 (128 x 256) are factored, each in a bucket of its own
    assert len(d1._factor) == 2 and not d2._factor
    torch.manual_seed(11)
    ref = ToyMLP(in_features=DIMS[0], hidden=DIMS[1], num_classes=10, device="cuda")
    ref.load_state_dict(m1.state_dict())
    ropt = (torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9) if opt_name == "sgd"
            else torch.optim.Adam(ref.parameters(), lr=1e-3))
    for i in range(5):
        x = torch.randn(64, DIMS[0], device="cuda")
        y = torch.randint(0, 10, (64,), device="cuda")
        for d, o in ((d1, o1), (d2, o2)):
            o.zero_grad(set_to_none=True)
            tdp.ops.cross_entropy(d(x), y).backward()
            o.step()
        _torch_step(ref, ropt, x, y)
        if i == 2:
            for o in (o1, o2, ropt):
                o.param_groups[0]["lr"] *= 0.5
    torch.cuda.synchronize()
    assert set(d1._factor_last_B.values()) == {64}
    for a, b, r in zip(m1.parameters(), m2.parameters(), ref.parameters()):
        torch.testing.assert_close(a, b, atol=2e-6, rtol=1e-5)
        torch.testing.assert_close(a, r, atol=2e-5, rtol=1e-4)
    # optimizer state of the factored weights matches the bucket path's
    s1, s2 = o1.state_dict()["state"], o2.state_dict()["state"]
    for k in s1:
        for name, v in s1[k].items():
            if torch.is_tensor(v) and v.numel() > 1:
                torch.testing.assert_close(v, s2[k][name], atol=2e-6, rtol=1e-5)


def test_factored_captured_step(pg):
    """The factored buckets inside a captured hipGraph step replay like eager steps."""
    tdp = pg
    from tutorial_torch_distributed_data_parallel_amd.train.graph import CapturedStep

    m1, d1, o1 = _build(tdp, "sgd", True, seed=5)
    m2, d2, o2 = _build(tdp, "sgd", True, seed=5)
    X = torch.randn(256, DIMS[0], device="cuda")
    Y = torch.randint(0, 10, (256,), device="cuda")
    idx = torch.zeros(32, dtype=torch.long, device="cuda")

    def make(d, o):
        def step():
            x, y = X.index_select(0, idx), Y.index_select(0, idx)
            o.zero_grad(set_to_none=True)
            loss = tdp.ops.cross_entropy(d(x), y)
            loss.backward()
            o.step()
            return loss
        return step

    eager = make(d1, o1)
    orders = [torch.randperm(256, device="cuda")[:32] for _ in range(7)]
    idx.copy_(orders[0])
    for _ in range(3):
        eager()
    graph = CapturedStep(make(d2, o2), warmup=3)
    for o in orders[1:]:
        idx.copy_(o)
        le, lg = eager(), graph.replay()
        torch.testing.assert_close(lg, le, atol=1e-5, rtol=1e-5)
    for a, b in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-4)


def test_early_prev_g_gather_captured_bitwise(pg, monkeypatch):
    """fc1's g gather issued from fc2's backward (right after fc2's gated input-gradient GEMM,
    ops/linear.py) instead of from fc1's own: the captured steps are bitwise identical to the
    ones without it, and fc1's own backward finds its gather already issued."""
    tdp = pg
    import importlib

    linear = importlib.import_module("tutorial_torch_distributed_data_parallel_amd.ops.linear")
    from tutorial_torch_distributed_data_parallel_amd.parallel.ddp import DistributedDataParallel
    from tutorial_torch_distributed_data_parallel_amd.train.graph import CapturedStep

    calls = []
    orig = DistributedDataParallel.factor_prefetch_g

    def spy(self, p, g):
        r = orig(self, p, g)
        calls.append((id(p), g.data_ptr(), r))
        return r

    monkeypatch.setattr(DistributedDataParallel, "factor_prefetch_g", spy)
    X = torch.randn(256, DIMS[0], device="cuda")
    Y = torch.randint(0, 10, (256,), device="cuda")
    idx = torch.zeros(32, dtype=torch.long, device="cuda")
    runs, counts = [], []
    for early in (True, False):
        old = linear.set_early_prev_g(early)
        try:
            m, d, o = _build(tdp, "sgd", True, seed=5)
            fc1 = id(m.fc1.weight)

            def step():
                x, y = X.index_select(0, idx), Y.index_select(0, idx)
                o.zero_grad(set_to_none=True)
                loss = tdp.ops.cross_entropy(d(x), y)
                loss.backward()
                o.step()
                return loss

            calls.clear()
            idx.zero_()  # the same warm-up batches in both runs
            graph = CapturedStep(step, warmup=3)
            n_fc1 = sum(1 for c in calls if c[0] == fc1 and c[2])
        finally:
            linear.set_early_prev_g(old)
        counts.append(n_fc1)
        torch.manual_seed(3)
        losses = []
        for _ in range(6):
            idx.copy_(torch.randperm(256, device="cuda")[:32])
            losses.append(graph.replay().clone())
        torch.cuda.synchronize()
        runs.append((torch.stack(losses), [p.detach().clone() for p in m.parameters()]))
    # warmup + capture: fc1's gather is asked for twice per step when early (fc2's backward,
    # then its own, which finds it issued), once otherwise
    assert counts[1] >= 1 and counts[0] == 2 * counts[1], counts
    assert torch.equal(runs[0][0], runs[1][0])
    for a, b in zip(runs[0][1], runs[1][1]):
        assert torch.equal(a, b)


def test_factored_skips_when_not_profitable(pg):
    """A batch too large for the factors to be cheaper than the gradient falls back to the
    ordinary weight-gradient GEMM (and the bucket's normal collectives)."""
    tdp = pg
    m1, d1, o1 = _build(tdp, "sgd", True, seed=6)
    m2, d2, o2 = _build(tdp, "sgd", False, seed=6)
    x = torch.randn(512, DIMS[0], device="cuda")  # 2*B*(out+in) > out*in for both layers
    y = torch.randint(0, 10, (512,), device="cuda")
    for d, o in ((d1, o1), (d2, o2)):
        o.zero_grad(set_to_none=True)
        tdp.ops.cross_entropy(d(x), y).backward()
        o.step()
    assert not d1._factor_last_B
    for a, b in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a, b, atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("opt_name", ["sgd", "adam"])
def test_replicated_factored_update_matches_sharded(pg, opt_name):
    """FactorJob.replicate: every rank computes all rows of the averaged gradient and updates
    them itself (no parameter all-gather). Rehearsed at world size 1 (where the shard is the
    whole weight) it must train like the sharded job: the weight rows are the same GEMM; the
    replicated job takes the bias gradient from that GEMM's row sums (its optimizer epilogue
    updates the bias) where the sharded job runs a column reduction, so the two agree to fp32
    rounding, not bit for bit. The auto policy picks it for W*B <= 768 only."""
    tdp = pg
    m1, d1, o1 = _build(tdp, opt_name, True, seed=21)
    m2, d2, o2 = _build(tdp, opt_name, True, seed=21)
    d1.factor_replicate, d2.factor_replicate = True, False
    for _ in range(4):
        x = torch.randn(64, DIMS[0], device="cuda")
        y = torch.randint(0, 10, (64,), device="cuda")
        for d, o in ((d1, o1), (d2, o2)):
            o.zero_grad(set_to_none=True)
            tdp.ops.cross_entropy(d(x), y).backward()
            o.step()
    torch.cuda.synchronize()
    assert set(d1._factor_last_B.values()) == {64}
    for a, b in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a, b, atol=1e-6, rtol=1e-5)
    assert d1._replicate_pays(2, 128) and d1._replicate_pays(4, 128)
    assert not d1._replicate_pays(8, 128) and d1._replicate_pays(1, 128)
