"""MI355X: the production optimizer paths against torch.optim + torch.nn.functional (fp32).

* the headline shapes (toy MLP 9216 -> 4096 -> 4096 -> 10, B = 128) through the world-size-1
  optimizer-in-wgrad-epilogue path, for every SGD / Adam epilogue variant (gemm_f32_set_opt_variant) with
  the persistent grid on and off (VERDICT r1 "weak" 1);
* a hipGraph-captured step with Adam and an LR change mid-run == the eager step (device hyper
  blocks: csrc/kernels.h HyperSlot);
* a parameter used twice in one forward;
* gradient clipping: native clip_grad_norm_, the in-reduction global clip, the per-rank clip.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DIMS = (9216, 4096, 4096, 10)


@pytest.fixture(scope="module")
def pg():
    import tutorial_torch_distributed_data_parallel_amd as tdp

    if not tdp.parallel.is_initialized():
        tdp.init_process_group("nccl", rank=0, world_size=1, local_rank=0)
    yield tdp
    tdp.destroy_process_group()


def _ref_forward(params, x):
    """fp32 torch reference of ToyMLP: params in module order [w1, b1, w2, b2, w3, b3]."""
    w1, b1, w2, b2, w3, b3 = params
    h = torch.relu(F.linear(x, w1, b1))
    h = torch.relu(F.linear(h, w2, b2))
    return F.linear(h, w3, b3)


def _batches(n, B=128, seed=11):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return [(torch.randn(B, DIMS[0], device="cuda", generator=g),
             torch.randint(0, 10, (B,), device="cuda", generator=g)) for _ in range(n)]


_REF_CACHE = {}


def _reference(kind, init, batches, lr_change_at):
    key = kind
    if key in _REF_CACHE:
        return _REF_CACHE[key]
    params = [t.clone().requires_grad_(True) for t in init]
    opt = (torch.optim.SGD(params, lr=0.01, momentum=0.9) if kind == "sgd"
           else torch.optim.Adam(params, lr=1e-4))
    for i, (x, y) in enumerate(batches):
        if i == lr_change_at:
            opt.param_groups[0]["lr"] *= 0.5
        opt.zero_grad(set_to_none=True)
        F.cross_entropy(_ref_forward(params, x), y).backward()
        opt.step()
    out = [p.detach().clone() for p in params]
    _REF_CACHE[key] = out
    return out


SGD_VARIANTS = [(v, persist) for v in (0, 4, 8, 12, 16, 24, 28, 88) for persist in (1, 0)]
ADAM_VARIANTS = [(v, persist) for v in (0, 16, 24, 28, 88) for persist in (1, 0)]


@pytest.mark.parametrize("kind,variant,persist",
                         [("sgd", v, p) for v, p in SGD_VARIANTS] +
                         [("adam", v, p) for v, p in ADAM_VARIANTS])
def test_headline_epilogue_variants_match_torch(pg, kind, variant, persist, monkeypatch):
    tdp = pg
    C = tdp._native.native()
    from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP

    monkeypatch.setenv("TDP_OPT_EPILOGUE", "1")
    old = C.gemm_f32_set_opt_variant()
    try:
        if kind == "sgd":
            C.gemm_f32_set_opt_variant(sgd=variant, persist=persist)
        else:
            C.gemm_f32_set_opt_variant(adam=variant, persist=persist)
        torch.manual_seed(21)
        model = ToyMLP(in_features=DIMS[0], hidden=DIMS[1:3], num_classes=DIMS[3],
                       device="cuda")
        init = [p.detach().clone() for p in model.parameters()]
        ddp = tdp.DDP(model, device_ids=[0])
        opt = (tdp.optim.SGD(ddp.parameters(), lr=0.01, momentum=0.9) if kind == "sgd"
               else tdp.optim.Adam(ddp.parameters(), lr=1e-4))
        assert ddp.register_fused_optimizer(opt) and ddp._epi_on
        batches = _batches(5)
        for i, (x, y) in enumerate(batches):
            if i == 3:
                opt.param_groups[0]["lr"] *= 0.5
            opt.zero_grad(set_to_none=True)
            tdp.ops.cross_entropy(ddp(x), y).backward()
            opt.step()
        torch.cuda.synchronize()
        ref = _reference(kind, init, batches, 3)
        for (n, p), r in zip(model.named_parameters(), ref):
            d = (p.detach() - r).abs()
            if kind == "sgd":
                torch.testing.assert_close(p.detach(), r, atol=2e-5, rtol=1e-4,
                                           msg=lambda m: f"{n}: {m}")
            else:
                # Adam normalises each gradient element: elements whose gradient is ~0 move by
                # up to lr per step on summation-order noise alone -> bound max and mean
                assert float(d.max()) < 5 * 1e-4, (n, float(d.max()))
                assert float(d.mean()) < 2e-6, (n, float(d.mean()))
    finally:
        C.gemm_f32_set_opt_variant(*old)


@pytest.mark.parametrize("kind", ["sgd", "adam"])
@pytest.mark.parametrize("hidden,captured", [((4096, 4096), False), ((4096, 4096), True),
                                             ((4096,), False)])
def test_paired_wgrad_launch_is_bitwise(pg, kind, hidden, captured, monkeypatch):
    """World size 1: consecutive weight-gradient + optimizer GEMMs held back and run as ONE
    persistent launch (bindings.cpp gemm_f32_opt hold, gemm_f32_fast_run_pair) give the same
    parameters, bitwise, as one launch each -- eager and hipGraph-captured; with one hidden layer
    the held GEMM runs alone at the end of backward (SyncBackend::wait_all)."""
    tdp = pg
    from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP
    import importlib

    from tutorial_torch_distributed_data_parallel_amd.train.graph import CapturedStep

    L = importlib.import_module("tutorial_torch_distributed_data_parallel_amd.ops.linear")

    monkeypatch.setenv("TDP_OPT_EPILOGUE", "1")
    batches = _batches(6)
    out = {}
    for pair in (False, True):
        old = L.set_pair_wgrad(pair)
        try:
            torch.manual_seed(5)
            model = ToyMLP(in_features=DIMS[0], hidden=hidden, num_classes=10, device="cuda")
            init = [p.detach().clone() for p in model.parameters()]
            ddp = tdp.DDP(model, device_ids=[0])
            opt = (tdp.optim.SGD(ddp.parameters(), lr=0.01, momentum=0.9) if kind == "sgd"
                   else tdp.optim.Adam(ddp.parameters(), lr=1e-4))
            assert ddp.register_fused_optimizer(opt) and ddp._epi_on
            xb = torch.empty_like(batches[0][0])
            yb = torch.empty_like(batches[0][1])

            def step():
                opt.zero_grad(set_to_none=True)
                tdp.ops.cross_entropy(ddp(xb), yb).backward()
                opt.step()

            if captured:
                xb.copy_(batches[0][0]); yb.copy_(batches[0][1])
                g = CapturedStep(step, warmup=1)  # warmup step = batch 0
                for x, y in batches[1:]:
                    xb.copy_(x); yb.copy_(y)
                    g.replay()
            else:
                for x, y in batches:
                    xb.copy_(x); yb.copy_(y)
                    step()
            torch.cuda.synchronize()
            out[pair] = [p.detach().clone() for p in model.parameters()]
        finally:
            L.set_pair_wgrad(old)
    for (n, _), a, b, p0 in zip(model.named_parameters(), out[False], out[True], init):
        assert not torch.equal(a, p0), n  # every parameter was updated
        assert torch.equal(a, b), (n, float((a - b).abs().max()))


def test_captured_adam_with_lr_change_matches_eager(pg):
    """A hipGraph step (train/graph.py) with a fused Adam (world 1: optimizer in the wgrad
    epilogue) stays identical to the eager step over 12 steps with an LR change: the step count
    and bias corrections advance on the device, the LR reaches the kernels via the hyper block."""
    tdp = pg
    from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP
    from tutorial_torch_distributed_data_parallel_amd.train.graph import CapturedStep

    def build(fused):
        torch.manual_seed(3)
        m = ToyMLP(in_features=512, hidden=(512, 256), num_classes=10, device="cuda")
        d = tdp.DDP(m, device_ids=[0])
        o = tdp.optim.Adam(d.parameters(), lr=2e-3)
        if fused:
            assert d.register_fused_optimizer(o)
        return m, d, o

    X = torch.randn(1024, 512, device="cuda")
    Y = torch.randint(0, 10, (1024,), device="cuda")
    idx = torch.zeros(128, dtype=torch.long, device="cuda")

    def make_step(d, opt):
        def step():
            x, y = X.index_select(0, idx), Y.index_select(0, idx)
            opt.zero_grad(set_to_none=True)
            loss = tdp.ops.cross_entropy(d(x), y)
            loss.backward()
            opt.step()
            return loss
        return step

    for fused in (True, False):
        m1, d1, o1 = build(fused)
        m2, d2, o2 = build(fused)
        eager = make_step(d1, o1)
        orders = [torch.randperm(1024, device="cuda")[:128] for _ in range(13)]
        idx.copy_(orders[0])
        for _ in range(3):
            eager()
        graph = CapturedStep(make_step(d2, o2), warmup=3)
        for i, o in enumerate(orders[1:]):
            if i == 6:
                for opt in (o1, o2):
                    opt.param_groups[0]["lr"] *= 0.25
            idx.copy_(o)
            le = eager()
            lg = graph.replay()
            torch.testing.assert_close(lg, le, atol=1e-5, rtol=1e-5)
        for a, b in zip(m1.parameters(), m2.parameters()):
            torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-4)
        # the device step count advanced with every replay and state_dict reports it
        sd = o2.state_dict()
        assert int(next(iter(sd["state"].values()))["step"]) == 3 + 12


@pytest.mark.parametrize("fused", [False, True])
def test_shared_parameter_gpu(pg, fused):
    """a Linear applied twice. The gradient is the sum of both uses; with the
    fused optimizer the epilogue must not update the weight from one use's partial gradient."""
    tdp = pg

    class Twice(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.inp = tdp.nn.Linear(256, 512, relu=True, device="cuda")
            self.mid = tdp.nn.Linear(512, 512, relu=True, device="cuda")
            self.out = tdp.nn.Linear(512, 10, device="cuda")

        def forward(self, x):
            return self.out(self.mid(self.mid(self.inp(x))))

    torch.manual_seed(7)
    model = Twice()
    params = [p.detach().clone().requires_grad_(True) for p in model.parameters()]
    ddp = tdp.DDP(model, device_ids=[0])
    opt = tdp.optim.SGD(ddp.parameters(), lr=0.05, momentum=0.9)
    ropt = torch.optim.SGD(params, lr=0.05, momentum=0.9)
    if fused:
        assert ddp.register_fused_optimizer(opt)
    for _ in range(3):
        x = torch.randn(128, 256, device="cuda")
        y = torch.randint(0, 10, (128,), device="cuda")
        opt.zero_grad(set_to_none=True)
        tdp.ops.cross_entropy(ddp(x), y).backward()
        if not fused:
            names = [n for n, _ in model.named_parameters()]
            grads = {n: p.grad.clone() for n, p in model.named_parameters()}
        opt.step()
        ropt.zero_grad(set_to_none=True)
        w1, b1, w2, b2, w3, b3 = params
        h = torch.relu(F.linear(x, w1, b1))
        h = torch.relu(F.linear(torch.relu(F.linear(h, w2, b2)), w2, b2))
        F.cross_entropy(F.linear(h, w3, b3), y).backward()
        if not fused:
            for n, p in zip(names, params):
                torch.testing.assert_close(grads[n], p.grad, atol=1e-5, rtol=1e-4)
        ropt.step()
    for p, r in zip(model.parameters(), params):
        torch.testing.assert_close(p.detach(), r.detach(), atol=1e-5, rtol=1e-4)


def test_native_clip_grad_norm_matches_torch(pg):
    tdp = pg
    torch.manual_seed(0)
    ps = [torch.randn(n, device="cuda", requires_grad=True) for n in (1000, 37, 4096 * 3)]
    qs = [p.detach().clone().requires_grad_(True) for p in ps]
    for p, q in zip(ps, qs):
        g = torch.randn_like(p) * 3
        p.grad, q.grad = g.clone(), g.clone()
    n1 = tdp.nn.utils.clip_grad_norm_(ps, 1.5)
    n2 = torch.nn.utils.clip_grad_norm_(qs, 1.5)
    torch.testing.assert_close(n1, n2, atol=1e-4, rtol=1e-5)
    for p, q in zip(ps, qs):
        torch.testing.assert_close(p.grad, q.grad, atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("mode", ["global", "local", "global_rehearsal"])
def test_in_reduction_clip_gpu(pg, mode, monkeypatch):
    """World size 1: the fused optimizer with clipping (deferred update after the device-side
    norm), and the per-rank clip before aggregation (== global at one rank); global_rehearsal
    runs the collective path (TDP_FORCE_COLLECTIVE)."""
    tdp = pg
    from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP

    if mode == "global_rehearsal":
        monkeypatch.setenv("TDP_FORCE_COLLECTIVE", "1")
    torch.manual_seed(9)
    model = ToyMLP(in_features=512, hidden=(384, 256), num_classes=10, device="cuda")
    params = [p.detach().clone().requires_grad_(True) for p in model.parameters()]
    ddp = tdp.DDP(model, device_ids=[0], bucket_cap_mb=0.25)
    opt = tdp.optim.SGD(ddp.parameters(), lr=0.1, momentum=0.9)
    ropt = torch.optim.SGD(params, lr=0.1, momentum=0.9)
    if mode == "local":
        ddp.clip_grad_norm_before_aggregation(0.05)
        ddp.register_fused_optimizer(opt)
    else:
        ddp.register_fused_optimizer(opt, clip_grad_norm=0.05)
    assert not ddp._epi_on  # clipping needs the materialised gradient
    for _ in range(4):
        x = torch.randn(128, 512, device="cuda")
        y = torch.randint(0, 10, (128,), device="cuda")
        opt.zero_grad(set_to_none=True)
        tdp.ops.cross_entropy(ddp(x), y).backward()
        ropt.zero_grad(set_to_none=True)
        F.cross_entropy(_ref_forward(params, x), y).backward()
        n = torch.nn.utils.clip_grad_norm_(params, 0.05)
        assert float(n) > 0.05
        ropt.step()
        torch.testing.assert_close(ddp.last_grad_norm(), n, atol=1e-5, rtol=1e-4)
    for p, r in zip(model.parameters(), params):
        torch.testing.assert_close(p.detach(), r.detach(), atol=2e-5, rtol=1e-4)


def test_commbench_at_world1(pg):
    """parallel/commbench.py (bench.py diagnostics, scripts/rccl_sweep.py) runs end to end."""
    tdp = pg
    from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP
    from tutorial_torch_distributed_data_parallel_amd.parallel import commbench

    rows = commbench.collective_busbw([4096, 1 << 20], iters=2, warmup=1)
    assert len(rows) == 6 and all(r["ms"] > 0 for r in rows)
    m = ToyMLP(in_features=256, hidden=(128,), num_classes=10, device="cuda")
    d = tdp.DDP(m, device_ids=[0])
    assert commbench.ddp_comm_ms(d, iters=2, warmup=1) > 0


@pytest.mark.parametrize("fused", [False, True])
def test_bucket_rebuild_gpu(pg, fused):
    """Arena relayout from the observed ready order on the device path (RcclOps, optimizer
    epilogue offsets and state re-bound) keeps training identical to torch."""
    tdp = pg

    class Shuffled(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = tdp.nn.Linear(256, 512, relu=True, device="cuda")
            self.c = tdp.nn.Linear(512, 10, device="cuda")
            self.b = tdp.nn.Linear(512, 512, relu=True, device="cuda")

        def forward(self, x):
            return self.c(self.b(self.a(x)))

    torch.manual_seed(5)
    model = Shuffled()
    names = [n for n, _ in model.named_parameters()]
    params = {n: p.detach().clone().requires_grad_(True) for n, p in model.named_parameters()}
    ddp = tdp.DDP(model, device_ids=[0], bucket_cap_mb=0.001, first_bucket_cap_mb=0.001)
    opt = tdp.optim.Adam(ddp.parameters(), lr=1e-3)
    ropt = torch.optim.Adam(params.values(), lr=1e-3)
    if fused:
        ddp.register_fused_optimizer(opt)
    for step in range(4):
        x = torch.randn(128, 256, device="cuda")
        y = torch.randint(0, 10, (128,), device="cuda")
        opt.zero_grad(set_to_none=True)
        tdp.ops.cross_entropy(ddp(x), y).backward()
        opt.step()
        ropt.zero_grad(set_to_none=True)
        P = params
        h = torch.relu(F.linear(x, P["a.weight"], P["a.bias"]))
        h = torch.relu(F.linear(h, P["b.weight"], P["b.bias"]))
        F.cross_entropy(F.linear(h, P["c.weight"], P["c.bias"]), y).backward()
        ropt.step()
        if step == 1:
            assert ddp._rebuilt
    for n, p in model.named_parameters():
        torch.testing.assert_close(p.detach(), params[n].detach(), atol=5e-5, rtol=1e-4,
                                   msg=lambda m: f"{n}: {m}")


@pytest.mark.gpu
def test_bench_diagnostics_deadline():
    """bench.py: diagnostics that overrun TDP_DIAG_TIMEOUT_S cannot cost the measurement -- the
    record is printed (one JSON line, diagnostics marked) and the process exits 0."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, TDP_DIAG_MULTI="1", TDP_DIAG_TIMEOUT_S="0.001")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--mlp-dims",
                        "256,128,128", "--steps", "3", "--warmup", "1", "--dataset", "512"],
                       env=env, capture_output=True, text=True, timeout=110, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["steps"] == 3 and rec["value"] > 0
    assert "exceeded" in rec["diagnostics"]["error"]


@pytest.mark.parametrize("kind", ["sgd", "adam"])
def test_fused_step_is_deterministic(pg, kind):
    """Two identical world-1 models with the fused optimizer (updates in the GEMM epilogues and
    in the one-launch head backward) stay BITWISE identical. Regression: the head backward's dx
    workgroups read W while its weight workgroups updated W in place -- a race that made
    identical models diverge from the first step (profiles/r8/diag_accel_hidden_r8f_before_fix.jsonl)."""
    tdp = pg
    from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP

    g = torch.Generator(device="cuda").manual_seed(7)
    data = [(torch.randn(64, 1024, device="cuda", generator=g),
             torch.randint(0, 10, (64,), device="cuda", generator=g)) for _ in range(6)]
    models = []
    for _ in range(2):
        torch.manual_seed(0)
        m = ToyMLP(in_features=1024, hidden=(512, 512), num_classes=10, device="cuda")
        d = tdp.DDP(m, device_ids=[0])
        o = (tdp.optim.SGD(d.parameters(), lr=0.05, momentum=0.9) if kind == "sgd"
             else tdp.optim.Adam(d.parameters(), lr=2e-3))
        assert d.register_fused_optimizer(o) and d._epi_on
        models.append((m, d, o))
    for i, (x, y) in enumerate(data):
        for m, d, o in models:
            if i == 3:
                o.param_groups[0]["lr"] *= 0.5
            o.zero_grad(set_to_none=True)
            tdp.ops.backward(tdp.ops.cross_entropy(d(x), y))
            o.step()
    torch.cuda.synchronize()
    for (n, a), b in zip(models[0][0].named_parameters(), models[1][0].parameters()):
        assert torch.equal(a, b), (n, float((a - b).abs().max()))
