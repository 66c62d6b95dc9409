"""MI355X: the Accelerate-style facade in ONE process (REF/multi-GPU-training-accelerate.py run
under plain python). ``prepare`` hands the module back unwrapped, as Accelerate does, but a
hidden world-1 DDP runs underneath so a fused optimizer can apply the update in the
weight-gradient GEMM epilogues: the step must equal the native DDP entry point's bitwise, and
gradient accumulation must still synchronise (and update) only on its last micro-step."""
import pytest
import torch
import torch.nn.functional as F

import tutorial_torch_distributed_data_parallel_amd as tdp
from tutorial_torch_distributed_data_parallel_amd.accelerate import Accelerator
from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP
from tutorial_torch_distributed_data_parallel_amd.parallel import runtime as rt

pytestmark = pytest.mark.gpu

DIMS = dict(in_features=1024, hidden=(512, 512), num_classes=10)


@pytest.fixture(scope="module")
def pg():
    if not rt.is_initialized():
        tdp.init_process_group("nccl", rank=0, world_size=1, local_rank=0)
    yield
    tdp.destroy_process_group()


def _batches(n, B=64):
    g = torch.Generator(device="cuda").manual_seed(7)
    return [(torch.randn(B, DIMS["in_features"], device="cuda", generator=g),
             torch.randint(0, 10, (B,), device="cuda", generator=g)) for _ in range(n)]


def test_one_process_accelerate_fused_matches_native_ddp(pg):
    data = _batches(6)
    torch.manual_seed(0)
    m1 = ToyMLP(**DIMS, device="cuda")
    torch.manual_seed(0)
    m2 = ToyMLP(**DIMS, device="cuda")
    d1 = tdp.DDP(m1, device_ids=[0])
    o1 = tdp.optim.SGD(d1.parameters(), lr=0.05, momentum=0.9)
    assert d1.register_fused_optimizer(o1) and d1._epi_on
    acc = Accelerator()
    o2 = tdp.optim.SGD(m2.parameters(), lr=0.05, momentum=0.9)
    model, opt = acc.prepare(m2, o2)
    assert model is m2 and not isinstance(model, tdp.DDP)  # unwrapped, like Accelerate
    assert acc.fuse_optimizer(model, opt) and acc.ddp_of(model)._epi_on
    for i, (x, y) in enumerate(data):
        if i == 3:
            for o in (o1, o2):
                o.param_groups[0]["lr"] *= 0.5
        o1.zero_grad(set_to_none=True)
        # the native entry point's backward (bench.py): seeded like accelerator.backward, so the
        # loss gradient comes from the same fused CE path
        tdp.ops.backward(tdp.ops.cross_entropy(d1(x), y))
        o1.step()
        opt.zero_grad(set_to_none=True)
        acc.backward(tdp.ops.cross_entropy(model(x), y))
        opt.step()
    torch.cuda.synchronize()
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        assert torch.equal(a, b), n
    assert set(model.state_dict()) == set(m1.state_dict())  # no "module." prefix


def test_one_process_accelerate_accumulation_with_fused_optimizer(pg):
    """GA = 2: the first micro-step of each window accumulates without any update, the second
    applies ONE update with the summed gradient -- the torch reference of the same schedule."""
    data = _batches(4)
    torch.manual_seed(0)
    m = ToyMLP(**DIMS, device="cuda")
    ref_params = [p.detach().clone().requires_grad_(True) for p in m.parameters()]
    acc = Accelerator(gradient_accumulation_steps=2)
    opt = tdp.optim.SGD(m.parameters(), lr=0.05, momentum=0.9)
    model, opt = acc.prepare(m, opt)
    assert acc.fuse_optimizer(model, opt)
    ropt = torch.optim.SGD(ref_params, lr=0.05, momentum=0.9)
    names = [n for n, _ in m.named_parameters()]
    P = dict(zip(names, ref_params))

    def ref_forward(x):
        h = torch.relu(F.linear(x, P["fc1.weight"], P["fc1.bias"]))
        h = torch.relu(F.linear(h, P["fc2.weight"], P["fc2.bias"]))
        return F.linear(h, P["fc3.weight"], P["fc3.bias"])

    for i, (x, y) in enumerate(data):
        with acc.accumulate(model):
            acc.backward(tdp.ops.cross_entropy(model(x), y))
            opt.step()
            opt.zero_grad(set_to_none=True)
        (F.cross_entropy(ref_forward(x), y) / 2).backward()
        if i % 2 == 1:
            ropt.step()
            ropt.zero_grad(set_to_none=True)
    torch.cuda.synchronize()
    for n, p in m.named_parameters():
        torch.testing.assert_close(p.detach(), P[n].detach(), atol=2e-5, rtol=1e-4,
                                   msg=lambda s: f"{n}: {s}")
