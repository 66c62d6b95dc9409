"""tdp optimizers on CPU tensors: torch.optim semantics of step hooks, zero_grad and LR
schedulers survive the lean step wrapper (optim/fused.py ``_lean_step_hook``)."""
import warnings

import torch

import tutorial_torch_distributed_data_parallel_amd as tdp


def _model():
    torch.manual_seed(0)
    return torch.nn.Linear(4, 3)


def test_step_hooks_and_zero_grad():
    m = _model()
    opt = tdp.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    calls = []
    h1 = opt.register_step_pre_hook(lambda o, a, k: calls.append("pre"))
    h2 = opt.register_step_post_hook(lambda o, a, k: calls.append("post"))
    m(torch.randn(2, 4)).sum().backward()
    opt.step()
    assert calls == ["pre", "post"]
    h1.remove(), h2.remove()
    opt.zero_grad()
    assert all(p.grad is None for p in m.parameters())
    m(torch.randn(2, 4)).sum().backward()
    opt.step()
    assert calls == ["pre", "post"]  # removed hooks are not called
    opt.zero_grad(set_to_none=False)
    assert all(torch.count_nonzero(p.grad) == 0 for p in m.parameters())


def test_matches_torch_sgd_and_adam_with_scheduler():
    for ours, ref in ((tdp.optim.SGD, torch.optim.SGD), (tdp.optim.Adam, torch.optim.Adam)):
        ma, mb = _model(), _model()
        kw = dict(lr=0.05, momentum=0.9) if ref is torch.optim.SGD else dict(lr=0.01)
        oa, ob = ours(ma.parameters(), **kw), ref(mb.parameters(), **kw)
        with warnings.catch_warnings():
            warnings.simplefilter("error")  # "lr_scheduler.step() before optimizer.step()" etc.
            sa = torch.optim.lr_scheduler.StepLR(oa, step_size=2, gamma=0.5)
            sb = torch.optim.lr_scheduler.StepLR(ob, step_size=2, gamma=0.5)
            x = torch.randn(8, 4)
            for _ in range(5):
                for m, o, s in ((ma, oa, sa), (mb, ob, sb)):
                    o.zero_grad()
                    m(x).pow(2).sum().backward()
                    o.step()
                    s.step()
        for pa, pb in zip(ma.parameters(), mb.parameters()):
            torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-6)
        assert oa.param_groups[0]["lr"] == ob.param_groups[0]["lr"]


def test_profiler_sees_optimizer_step():
    m = _model()
    opt = tdp.optim.SGD(m.parameters(), lr=0.1)
    m(torch.randn(2, 4)).sum().backward()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        opt.step()
    names = {e.name for e in prof.events()}
    assert any(n.startswith("Optimizer.step#SGD.step") for n in names), names


def test_dense_views_follow_storage_order():
    """The multi-tensor kernels see p, grad and state as 1-D views in the PARAMETER's storage
    order: channels_last conv weights stay views (no copy), a gradient of the other layout is
    converted to the parameter's order."""
    from tutorial_torch_distributed_data_parallel_amd.optim.fused import _dense, _grad_like

    w = torch.randn(4, 3, 2, 2).contiguous(memory_format=torch.channels_last)
    w.grad = torch.randn(4, 3, 2, 2)  # plain contiguous gradient
    v = _dense(w)
    assert v.data_ptr() == w.data_ptr() and v.dim() == 1
    assert torch.equal(v, w.permute(0, 2, 3, 1).reshape(-1))
    assert torch.equal(_grad_like(w), w.grad.permute(0, 2, 3, 1).reshape(-1))
    b = torch.randn(5)
    b.grad = torch.randn(5)
    assert _dense(b).data_ptr() == b.data_ptr() and torch.equal(_grad_like(b), b.grad)
    try:
        _dense(torch.randn(4, 6)[:, ::2])
    except RuntimeError:
        pass
    else:
        raise AssertionError("strided tensors must be rejected")


def test_replicated_factored_update_price_model():
    """parallel/ddp.py: the replicated factored update is chosen for W*B <= 768 only (2 and 4
    ranks at the reference's per-rank batch of 128, never at eight; at one rank -- the one-GPU
    rehearsal -- replicating skips the in-place parameter all-gather)."""
    from tutorial_torch_distributed_data_parallel_amd.parallel.ddp import DistributedDataParallel

    pays = DistributedDataParallel._replicate_pays
    assert pays(2, 128) and pays(4, 128)
    assert pays(1, 128) and not pays(8, 128) and pays(8, 64)
