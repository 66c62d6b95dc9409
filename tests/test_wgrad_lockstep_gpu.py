"""MI355X: the lockstep weight-gradient + optimizer kernel (csrc/gemm_f32_fast.hip
wgrad_lockstep_kernel: math and stream waves of one workgroup on shared barriers; opt-in,
measured at parity with the default: profiles/r9/wgrad_split_roles_r9.md) against the persistent epilogue kernel,
the per-bucket fused update and plain optimizer.step() (torch semantics), on shapes with partial
128 x 128 tiles and K (batch) tails (which keep the persistent kernel); plus run-to-run bitwise
determinism."""
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


def _native():
    from tutorial_torch_distributed_data_parallel_amd._native import native

    return native()


def _build(tdp, dims, opt_name, mode, monkeypatch, seed=5):
    from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP

    monkeypatch.setenv("TDP_OPT_EPILOGUE", "0" if mode == "bucket" else "1")
    torch.manual_seed(seed)
    m = ToyMLP(in_features=dims[0], hidden=dims[1:], num_classes=10, device="cuda")
    d = tdp.DDP(m, device_ids=[0], bucket_cap_mb=0.5, first_bucket_cap_mb=0.02)
    if opt_name == "sgd":
        o = tdp.optim.SGD(d.parameters(), lr=0.05, momentum=0.9)
    elif opt_name == "sgd_nesterov_wd":
        o = tdp.optim.SGD(d.parameters(), lr=0.05, momentum=0.9, nesterov=True,
                          weight_decay=1e-3)
    elif opt_name == "adamw":
        o = tdp.optim.AdamW(d.parameters(), lr=1e-3, weight_decay=1e-2)
    else:
        o = tdp.optim.Adam(d.parameters(), lr=1e-3)
    if mode != "plain":
        assert d.register_fused_optimizer(o)
    return m, d, o


def _train(tdp, runs, dims, batch, steps=4):
    was = _native().gemm_f32_lockstep()
    g = torch.Generator(device="cuda").manual_seed(11)
    for i in range(steps):
        x = torch.randn(batch, dims[0], device="cuda", generator=g)
        y = torch.randint(0, 10, (batch,), device="cuda", generator=g)
        for _, d, o, ls in runs:
            _native().gemm_f32_set_lockstep(ls)  # read at every GEMM plan
            o.zero_grad(set_to_none=True)
            tdp.ops.cross_entropy(d(x), y).backward()
            o.step()
        if i == 1:
            for _, _, o, _ in runs:
                o.param_groups[0]["lr"] *= 0.5
    _native().gemm_f32_set_lockstep(was)
    torch.cuda.synchronize()


MODES = (("plain", True), ("bucket", True), ("epilogue (persistent)", False),
         ("epilogue (lockstep)", True))


@pytest.mark.parametrize("dims,batch", [((512, 384, 256), 128), ((260, 132, 388), 72),
                                        ((256, 128, 128), 8), ((512, 256, 384), 256)])
@pytest.mark.parametrize("opt_name", ["sgd", "sgd_nesterov_wd", "adam", "adamw"])
def test_split_role_epilogues_match_reference_paths(pg, dims, batch, opt_name, monkeypatch):
    tdp = pg
    runs = []
    for name, flags in MODES:
        mode = name.split()[0]
        m, d, o = _build(tdp, dims, opt_name, mode, monkeypatch)
        assert d._epi_on == (mode == "epilogue")
        runs.append((m, d, o, flags))
    _train(tdp, runs, dims, batch)
    atol = 2e-6
    for (m, _, _, _), (name, _) in zip(runs[1:], MODES[1:]):
        for (n, a), b in zip(runs[0][0].named_parameters(), m.parameters()):
            torch.testing.assert_close(b, a, atol=atol, rtol=1e-5,
                                       msg=lambda s: f"{name} {n}: {s}")
    # the lockstep kernel runs the persistent kernel's K loop: bit-identical
    for (n, a), b in zip(runs[2][0].named_parameters(), runs[3][0].parameters()):
        assert torch.equal(a, b), f"{n}: lockstep != persistent epilogue"


def test_lockstep_epilogue_is_deterministic(pg, monkeypatch):
    """Two identical fused runs end bit-identical (no read / update race between the roles)."""
    tdp = pg
    dims = (1024, 768, 512)
    runs = []
    for _ in range(2):
        m, d, o = _build(tdp, dims, "sgd", "epilogue", monkeypatch)
        runs.append((m, d, o, True))
    _train(tdp, runs, dims, 128, steps=6)
    for a, b in zip(runs[0][0].parameters(), runs[1][0].parameters()):
        assert torch.equal(a, b)
