"""MI355X: the warp-specialised weight-gradient + optimizer kernel (csrc/gemm_wgrad_opt.hip) --
the default optimizer epilogue at world size 1 -- against the persistent epilogue kernel it
replaces, the per-bucket fused update and plain optimizer.step() (torch semantics), on shapes
with partial 128 x 128 tiles and a K (batch) tail; plus run-to-run bitwise determinism."""
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
    was = _native().wgrad_opt_enabled()
    g = torch.Generator(device="cuda").manual_seed(11)
    for i in range(steps):
        x = torch.randn(batch, dims[0], device="cuda", generator=g)
        y = torch.randint(0, 10, (batch,), device="cuda", generator=g)
        for _, d, o, ws in runs:
            _native().wgrad_opt_set_enabled(ws)  # read at every GEMM plan
            o.zero_grad(set_to_none=True)
            tdp.ops.cross_entropy(d(x), y).backward()
            o.step()
        if i == 1:
            for _, _, o, _ in runs:
                o.param_groups[0]["lr"] *= 0.5
    _native().wgrad_opt_set_enabled(was)
    torch.cuda.synchronize()


@pytest.mark.parametrize("dims,batch", [((512, 384, 256), 128), ((260, 132, 388), 72),
                                        ((256, 128, 128), 8)])
@pytest.mark.parametrize("opt_name", ["sgd", "sgd_nesterov_wd", "adam", "adamw"])
def test_ws_epilogue_matches_reference_paths(pg, dims, batch, opt_name, monkeypatch):
    tdp = pg
    runs = []
    for mode, ws in (("plain", True), ("bucket", True), ("epilogue", False), ("epilogue", True)):
        m, d, o = _build(tdp, dims, opt_name, mode, monkeypatch)
        assert d._epi_on == (mode == "epilogue")
        runs.append((m, d, o, ws))
    _train(tdp, runs, dims, batch)
    ref = list(runs[0][0].parameters())
    atol = 2e-6
    for (m, _, _, ws), mode in zip(runs[1:], ("bucket", "epilogue (persistent)",
                                              "epilogue (warp-specialised)")):
        for (n, a), b in zip(runs[0][0].named_parameters(), m.parameters()):
            torch.testing.assert_close(b, a, atol=atol, rtol=1e-5,
                                       msg=lambda s: f"{mode} {n}: {s}")
    # same MFMA operands in the same k slots, same row-sum order: bit-identical to the kernel
    # it replaces
    for (n, a), b in zip(runs[2][0].named_parameters(), runs[3][0].parameters()):
        assert torch.equal(a, b), f"{n}: warp-specialised != persistent epilogue"


def test_ws_epilogue_is_deterministic(pg, monkeypatch):
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
