"""MI355X: the fused head + cross-entropy op (ops.linear_cross_entropy, csrc/gemm_skinny.hip
head_ce_kernel) against the unfused native ops it replaces (skinny GEMM + ce_fwd + head_bwd:
bit for bit) and against the fp32 torch oracle; the toy MLP's training step through it (eager
and captured, DDP with the optimizer in the GEMM epilogues) equals the unfused step bit for
bit."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _native():
    from tutorial_torch_distributed_data_parallel_amd._native import native

    return native()


@pytest.mark.parametrize("B,O,I,smooth,ignore", [(128, 10, 4096, 0.0, False),
                                                  (64, 10, 1024, 0.1, True),
                                                  (200, 7, 512, 0.0, False),
                                                  (32, 16, 2048, 0.0, True)])
def test_head_ce_matches_unfused_ops_bitwise(B, O, I, smooth, ignore):
    from tutorial_torch_distributed_data_parallel_amd.ops.loss import _ticket

    C = _native()
    torch.manual_seed(B + O)
    x = torch.relu(torch.randn(B, I, device="cuda"))
    w = torch.randn(O, I, device="cuda") * 0.05
    b = torch.randn(O, device="cuda")
    y = torch.randint(0, O, (B,), device="cuda")
    if ignore:
        y[::5] = -100
    acc1 = torch.zeros(3, device="cuda")
    acc2 = torch.zeros(3, device="cuda")
    for _ in range(2):  # the ticket is zero again after every launch
        out = C.head_ce(x, w, b, y, -100, smooth, True, acc1, with_grad=True, gate=x,
                        planes=True, ticket=_ticket(x.device))
    loss, lse, logits, d, dx, pl = out
    # unfused: skinny head GEMM, ce_fwd with its unit-seed gradient, head_bwd's input gradient
    lg = torch.empty(B, O, device="cuda")
    C.gemm_f32(x, w, lg, True, True, bias=b)
    ref = None
    for _ in range(2):
        ref = C.ce_fwd(lg, y, -100, smooth, True, acc2, with_grad=True)
    dx2 = torch.empty_like(x)
    dw = torch.empty_like(w)
    ok, pl2 = C.head_bwd(ref[2], x, w, dx2, dw, gate=x, planes=True)
    torch.cuda.synchronize()
    assert ok
    assert torch.equal(logits, lg)
    assert torch.equal(loss, ref[0]) and torch.equal(lse, ref[1]) and torch.equal(d, ref[2])
    assert torch.equal(acc1, acc2), (acc1, acc2)
    assert torch.equal(dx, dx2) and torch.equal(pl, pl2)
    # and the fp32 oracle
    want = F.cross_entropy(x @ w.t() + b, y, ignore_index=-100, label_smoothing=smooth)
    torch.testing.assert_close(loss, want, rtol=1e-5, atol=1e-5)


def test_linear_cross_entropy_autograd_and_scaled_seed():
    """Gradients of the fused op == autograd through torch ops (fp32), for the unit seed (the
    forward's precomputed dlogits / dx) and a scaled seed (the unfused backward path)."""
    import tutorial_torch_distributed_data_parallel_amd as tdp

    torch.manual_seed(3)
    x0 = torch.relu(torch.randn(128, 1024, device="cuda"))
    w0 = torch.randn(10, 1024, device="cuda") * 0.05
    b0 = torch.randn(10, device="cuda")
    y = torch.randint(0, 10, (128,), device="cuda")
    for scale in (1.0, 0.25):
        x = x0.clone().requires_grad_()
        w = w0.clone().requires_grad_()
        b = b0.clone().requires_grad_()
        loss = tdp.ops.linear_cross_entropy(x, w, b, y)
        tdp.ops.backward(loss, scale)
        xr = x0.clone().requires_grad_()
        wr = w0.clone().requires_grad_()
        br = b0.clone().requires_grad_()
        (F.cross_entropy(xr @ wr.t() + br, y) * scale).backward()
        torch.testing.assert_close(loss, F.cross_entropy(x0 @ w0.t() + b0, y), rtol=1e-5,
                                   atol=1e-5)
        torch.testing.assert_close(x.grad, xr.grad, rtol=1e-4, atol=1e-6)
        torch.testing.assert_close(w.grad, wr.grad, rtol=1e-4, atol=1e-6)
        torch.testing.assert_close(b.grad, br.grad, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("captured", [False, True])
def test_toy_mlp_step_fused_head_equals_unfused(captured):
    """The toy MLP under DDP (world size 1, fused SGD in the GEMM epilogues): ``model(x,
    target=y)`` and ``cross_entropy(model(x), y)`` give bit-identical parameters and metric sums
    after several steps, eager and as a replayed hipGraph."""
    import tutorial_torch_distributed_data_parallel_amd as tdp
    from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP
    from tutorial_torch_distributed_data_parallel_amd.parallel import runtime as rt
    from tutorial_torch_distributed_data_parallel_amd.train.graph import CapturedStep

    import os
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if not tdp.parallel.is_initialized():
        tdp.init_process_group("nccl", rank=0, world_size=1, local_rank=0)
    dev = rt.device()
    xs = [torch.randn(128, 1024, device=dev) for _ in range(4)]
    ys = [torch.randint(0, 10, (128,), device=dev) for _ in range(4)]
    res = []
    for fused in (True, False):
        torch.manual_seed(0)
        m = ToyMLP(in_features=1024, hidden=(512, 512), device=dev)
        ddp = tdp.DDP(m, device_ids=[dev.index])
        opt = tdp.optim.SGD(ddp.parameters(), lr=0.05, momentum=0.9)
        ddp.register_fused_optimizer(opt)
        acc = torch.zeros(3, device=dev)
        sx = torch.empty(128, 1024, device=dev)
        sy = torch.empty(128, dtype=torch.long, device=dev)

        def step():
            opt.zero_grad(set_to_none=True)
            if fused:
                loss = ddp(sx, target=sy, acc=acc)
            else:
                loss = tdp.ops.cross_entropy(ddp(sx), sy, acc=acc)
            tdp.ops.backward(loss)
            opt.step()
            return loss
        g = None
        for i in range(4):
            sx.copy_(xs[i])
            sy.copy_(ys[i])
            if not captured:
                step()
            elif g is None:
                g = CapturedStep(step, warmup=1)
            else:
                g.replay()
        torch.cuda.synchronize()
        res.append(([p.detach().clone() for p in m.parameters()], acc.clone()))
    (pf, af), (pu, au) = res
    for i, (a, b) in enumerate(zip(pf, pu)):
        assert torch.equal(a, b), f"param {i} differs (max {float((a - b).abs().max())})"
    assert torch.equal(af, au), (af, au)
