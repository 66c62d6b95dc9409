"""Numerics of every native gfx950 kernel against a plain PyTorch fp32 reference of the same op."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def C():
    from tutorial_torch_distributed_data_parallel_amd._native import native

    return native()


def _close(a, b, rtol=1e-4, atol=1e-4):
    torch.testing.assert_close(a, b, rtol=rtol, atol=atol)


def _ref_gemm(A, B, a_k, b_k, mask=None):
    Am = A if mask is None else torch.where(mask > 0, A, torch.zeros_like(A))
    A2 = Am if a_k else Am.t()
    B2 = B.t() if b_k else B
    return (A2.double() @ B2.double()).float()


SHAPES = [(128, 4096, 9216), (128, 10, 4096), (128, 4096, 10), (4096, 4096, 128),
          (10, 4096, 128), (37, 53, 71), (1, 1, 1), (256, 320, 96), (130, 66, 257),
          (132, 196, 100), (260, 136, 44), (64, 8, 4)]


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("a_k,b_k", [(True, True), (True, False), (False, False), (False, True)])
def test_gemm_layouts(C, M, N, K, a_k, b_k, mode):
    if M * N * K > 128 * 4096 * 9216 // 4 and not (a_k and b_k):
        pytest.skip("large shape covered in the forward layout")
    torch.manual_seed(M + N + K)
    d = "cuda"
    A = torch.randn((M, K) if a_k else (K, M), device=d)
    B = torch.randn((N, K) if b_k else (K, N), device=d)
    out = torch.empty(M, N, device=d)
    C.gemm_f32_set_mode(mode)  # 0: auto (LDS-DMA fast kernel when aligned), 1: generic
    try:
        C.gemm_f32(A, B, out, a_k, b_k)
    finally:
        C.gemm_f32_set_mode(0)
    ref = _ref_gemm(A, B, a_k, b_k)
    tol = 2e-4 * max(1.0, K ** 0.5)
    _close(out, ref, rtol=1e-4, atol=tol)


def test_gemm_asymmetric_identity(C):
    # A = I with an asymmetric B catches transposed C/D maps (guide §3)
    n = 64
    A = torch.eye(n, device="cuda")
    B = torch.arange(n * n, device="cuda", dtype=torch.float32).reshape(n, n) / 7.0
    out = torch.empty(n, n, device="cuda")
    C.gemm_f32(A, B, out, True, False)
    _close(out, B, rtol=0, atol=0)


def test_gemm_epilogues(C):
    torch.manual_seed(0)
    M, N, K = 96, 200, 300
    A = torch.randn(M, K, device="cuda")
    W = torch.randn(N, K, device="cuda")
    b = torch.randn(N, device="cuda")
    out = torch.empty(M, N, device="cuda")
    C.gemm_f32(A, W, out, True, True, bias=b, relu=True)
    ref = torch.relu(_ref_gemm(A, W, True, True) + b)
    _close(out, ref, atol=3e-3)
    # beta accumulate
    base = torch.randn(M, N, device="cuda")
    out2 = base.clone()
    C.gemm_f32(A, W, out2, True, True, beta=1.0)
    _close(out2, base + _ref_gemm(A, W, True, True), atol=3e-3)


def test_gemm_mask_and_rowsum(C):
    torch.manual_seed(1)
    Bt, out_f, in_f = 128, 192, 320
    dy = torch.randn(Bt, out_f, device="cuda")
    y = torch.relu(torch.randn(Bt, out_f, device="cuda"))
    x = torch.randn(Bt, in_f, device="cuda")
    dw = torch.empty(out_f, in_f, device="cuda")
    db = torch.empty(out_f, device="cuda")
    C.gemm_f32(dy, x, dw, False, False, mask=y, rowsum=db)
    g = dy * (y > 0)
    _close(dw, (g.t().double() @ x.double()).float(), atol=2e-3)
    _close(db, g.sum(0), atol=1e-3)


def test_ce_fwd_bwd(C):
    torch.manual_seed(2)
    for B, Cl in [(128, 10), (64, 1000), (7, 3)]:
        z = torch.randn(B, Cl, device="cuda", requires_grad=True)
        y = torch.randint(0, Cl, (B,), device="cuda")
        y[0] = -100
        for smooth in (0.0, 0.1):
            acc = torch.zeros(3, device="cuda")
            loss, lse = C.ce_fwd(z.detach(), y, -100, smooth, True, acc)
            ref = torch.nn.functional.cross_entropy(z, y, label_smoothing=smooth)
            _close(loss, ref.detach(), atol=1e-5)
            (gref,) = torch.autograd.grad(ref, z)
            d = C.ce_bwd(z.detach(), y, lse, torch.ones(1, device="cuda"), -100, smooth, True)
            _close(d, gref, atol=1e-6)
            valid = y != -100
            assert acc[2].item() == valid.sum().item()
            correct = ((z.argmax(1) == y) & valid).sum().item()
            assert acc[1].item() == correct


def test_sgd_flat_matches_torch(C):
    torch.manual_seed(3)
    n = 1000003
    for mom, nest, wd, damp in [(0.9, False, 0.0, 0.0), (0.9, True, 1e-4, 0.0),
                                (0.0, False, 1e-2, 0.0), (0.5, False, 0.0, 0.1)]:
        p = torch.randn(n, device="cuda")
        p_ref = p.clone().requires_grad_()
        opt = torch.optim.SGD([p_ref], lr=0.1, momentum=mom, nesterov=nest, weight_decay=wd,
                              dampening=damp)
        buf = torch.empty_like(p)
        for t in range(3):
            g = torch.randn(n, device="cuda")
            p_ref.grad = g.clone()
            opt.step()
            C.sgd_flat(p, g, buf if mom else None, 0.1, mom, damp, wd, nest, False, t == 0, 1.0)
        _close(p, p_ref.detach(), atol=1e-5)


def test_adam_flat_matches_torch(C):
    torch.manual_seed(4)
    n = 500001
    for wd, ams, decoupled in [(0.0, False, False), (1e-2, True, False), (1e-2, False, True)]:
        p = torch.randn(n, device="cuda")
        p_ref = p.clone().requires_grad_()
        cls = torch.optim.AdamW if decoupled else torch.optim.Adam
        opt = cls([p_ref], lr=1e-3, weight_decay=wd, amsgrad=ams)
        m, v, vm = (torch.zeros_like(p) for _ in range(3))
        for t in range(1, 4):
            g = torch.randn(n, device="cuda")
            p_ref.grad = g.clone()
            opt.step()
            C.adam_flat(p, g, m, v, vm if ams else None, 1e-3, 0.9, 0.999, 1e-8, wd, ams, False,
                        decoupled, t, 1.0)
        _close(p, p_ref.detach(), atol=1e-6, rtol=1e-5)


def test_multi_tensor_sgd_adam(C):
    torch.manual_seed(5)
    shapes = [(3, 5), (70000,), (128, 129), (1,)]
    ps = [torch.randn(s, device="cuda") for s in shapes]
    gs = [torch.randn(s, device="cuda") for s in shapes]
    bufs = [torch.empty_like(p) for p in ps]
    refs = [p.clone().requires_grad_() for p in ps]
    opt = torch.optim.SGD(refs, lr=0.05, momentum=0.9)
    for r, g in zip(refs, gs):
        r.grad = g.clone()
    opt.step()
    C.sgd_multi(ps, gs, bufs, 0.05, 0.9, 0.0, 0.0, False, False, True, 1.0)
    for p, r in zip(ps, refs):
        _close(p, r.detach(), atol=1e-6)


@pytest.mark.parametrize("shape", [(128, 4096), (32, 64, 7, 7), (5, 3), (8, 16, 33), (1000, 64),
                                   (300, 2048), (77, 12), (6000, 256)])
def test_batchnorm_kernels(C, shape):
    torch.manual_seed(6)
    x = torch.randn(shape, device="cuda") * 3 + 1
    Cn = shape[1]
    w = torch.randn(Cn, device="cuda")
    b = torch.randn(Cn, device="cuda")
    st = C.bn_moments(x)[0]
    dims = [0] + list(range(2, x.dim()))
    _close(st[:Cn], x.mean(dims), atol=1e-5)
    _close(st[Cn:2 * Cn], x.var(dims, unbiased=False), atol=1e-4, rtol=1e-4)
    rm, rv = torch.zeros(Cn, device="cuda"), torch.ones(Cn, device="cuda")
    stats = C.bn_merge(st, Cn, 1e-5, 0.1, rm, rv)
    xr = x.clone().requires_grad_()
    wr, br = w.clone().requires_grad_(), b.clone().requires_grad_()
    rm2, rv2 = torch.zeros(Cn, device="cuda"), torch.ones(Cn, device="cuda")
    yref = torch.relu(torch.nn.functional.batch_norm(xr, rm2, rv2, wr, br, True, 0.1, 1e-5))
    y = C.bn_elemt(x, stats, w, b, True)
    _close(y, yref.detach(), atol=1e-4)
    _close(rm, rm2, atol=1e-5)
    _close(rv, rv2, atol=1e-4)
    dy = torch.randn_like(x)
    gx, gw, gb = torch.autograd.grad(yref, (xr, wr, br), dy)
    dw, db = torch.empty_like(w), torch.empty_like(b)
    sums = C.bn_bwd_reduce(dy, x, stats, y, dw, db, 0.0)
    dx = C.bn_bwd_elemt(dy, x, stats, w, sums, y)[0]
    _close(dw, gw, atol=1e-3, rtol=1e-4)
    _close(db, gb, atol=1e-3, rtol=1e-4)
    _close(dx, gx, atol=1e-4, rtol=1e-4)
    ye = C.bn_eval(x, rm, rv, w, b, 1e-5, False)
    _close(ye, torch.nn.functional.batch_norm(x, rm, rv, w, b, False, 0.0, 1e-5), atol=1e-4)


@pytest.mark.parametrize("shape", [(128, 4096), (6000, 256), (77, 12), (300, 2048)])
def test_batchnorm_relu_mask_path(C, shape):
    """csrc/norm.hip: the forward's 1-byte-per-4-channels ReLU mask (bit j = channel 4q+j > 0)
    drives the backward exactly as the float output does."""
    torch.manual_seed(11)
    x = torch.randn(shape, device="cuda") * 2 + 0.3
    Cn = shape[1]
    w, b = torch.randn(Cn, device="cuda"), torch.randn(Cn, device="cuda")
    res = torch.randn(shape, device="cuda")
    st = C.bn_moments(x)[0]
    stats = C.bn_merge(st, Cn, 1e-5, 0.1, None, None)
    mask = torch.empty((shape[0], Cn // 4), dtype=torch.uint8, device="cuda")
    y = C.bn_elemt(x, stats, w, b, True, res, mask_out=mask)
    y_ref = C.bn_elemt(x, stats, w, b, True, res)
    assert torch.equal(y, y_ref)
    bits = (y > 0).view(shape[0], Cn // 4, 4).to(torch.int32)
    packed = (bits * torch.tensor([1, 2, 4, 8], device="cuda", dtype=torch.int32)).sum(-1)
    assert torch.equal(mask.to(torch.int32), packed)
    dy = torch.randn(shape, device="cuda")
    dw1, db1, dw2, db2 = (torch.empty(Cn, device="cuda") for _ in range(4))
    s1 = C.bn_bwd_reduce(dy, x, stats, y, dw1, db1, 0.0)
    s2 = C.bn_bwd_reduce(dy, x, stats, None, dw2, db2, 0.0, mask=mask)
    assert torch.equal(s1, s2) and torch.equal(dw1, dw2) and torch.equal(db1, db2)
    o1 = C.bn_bwd_elemt(dy, x, stats, w, s1, y, True)
    o2 = C.bn_bwd_elemt(dy, x, stats, w, s2, None, True, mask=mask)
    assert torch.equal(o1[0], o2[0]) and torch.equal(o1[1], o2[1])


def test_linear_autograd_matches_torch():
    from tutorial_torch_distributed_data_parallel_amd import ops

    torch.manual_seed(7)
    x = torch.randn(128, 300, device="cuda", requires_grad=True)
    w = torch.randn(200, 300, device="cuda", requires_grad=True)
    b = torch.randn(200, device="cuda", requires_grad=True)
    dy = torch.randn(128, 200, device="cuda")
    for relu in (False, True):
        y = ops.linear(x, w, b, relu=relu)
        gx, gw, gb = torch.autograd.grad(y, (x, w, b), dy)
        yr = torch.nn.functional.linear(x.double(), w.double(), b.double())
        if relu:
            yr = torch.relu(yr)
        rgx, rgw, rgb = torch.autograd.grad(yr, (x, w, b), dy.double())
        _close(y, yr.float(), atol=2e-3)
        _close(gx, rgx.float(), atol=2e-3)
        _close(gw, rgw.float(), atol=2e-3)
        _close(gb, rgb.float(), atol=2e-3)


def test_gemm_fast_epilogue_and_split(C):
    torch.manual_seed(9)
    for (M, N, K) in [(128, 4096, 4096), (96, 200, 300), (200, 260, 1024)]:
        A = torch.randn(M, K, device="cuda")
        W = torch.randn(N, K, device="cuda")
        b = torch.randn(N, device="cuda")
        out = torch.empty(M, N, device="cuda")
        C.gemm_f32(A, W, out, True, True, bias=b, relu=True)
        ref = torch.relu(_ref_gemm(A, W, True, True) + b)
        _close(out, ref, atol=2e-4 * K ** 0.5)


def test_relu_bias_bwd(C):
    torch.manual_seed(10)
    # FC shapes, odd shapes, and conv outputs viewed as [pixels, Cout] (narrow channel counts
    # take the CGB < 64 block shapes, 48 channels = 12 float4 groups)
    for B, N in [(128, 4096), (37, 130), (5, 3), (60000, 64), (20000, 192), (3000, 384),
                 (4001, 48), (777, 20)]:
        dy = torch.randn(B, N, device="cuda")
        y = torch.relu(torch.randn(B, N, device="cuda"))
        db = torch.empty(N, device="cuda")
        g = C.relu_bias_bwd(dy, y, db)
        ref = dy * (y > 0)
        tol = 1e-4 * max(1.0, B ** 0.5)
        _close(g, ref, atol=0, rtol=0)
        _close(db, ref.double().sum(0).float(), atol=tol)
        db2 = torch.empty(N, device="cuda")
        g2 = C.relu_bias_bwd(dy, None, db2)
        assert g2.data_ptr() == dy.data_ptr()
        _close(db2, dy.double().sum(0).float(), atol=tol)
        db3 = torch.ones(N, device="cuda")
        C.relu_bias_bwd(dy, y, db3, 0.5)  # accumulate: db = 0.5 * db + sum
        _close(db3, 0.5 + ref.double().sum(0).float(), atol=tol)


def test_gemm_fast_wgrad_rowsum(C):
    """Bias gradient reduced inside the LDS-DMA wgrad kernel (A = g^T, MN-contiguous)."""
    torch.manual_seed(11)
    for B, out_f, in_f in [(128, 256, 384), (64, 132, 200), (128, 4096, 256)]:
        g = torch.randn(B, out_f, device="cuda")
        x = torch.randn(B, in_f, device="cuda")
        dw = torch.empty(out_f, in_f, device="cuda")
        db = torch.full((out_f,), 7.0, device="cuda")
        C.gemm_f32(g, x, dw, False, False, rowsum=db)
        _close(dw, (g.t().double() @ x.double()).float(), atol=2e-3)
        _close(db, g.sum(0), atol=1e-3)


@pytest.mark.parametrize("M,N,K,a_k,b_k", [(128, 10, 4096, True, True), (77, 13, 260, True, True),
                                           (50, 1, 64, True, True), (20, 9, 1000, True, True),
                                           (128, 4096, 10, True, False), (33, 64, 16, True, False),
                                           (10, 4096, 128, False, False), (16, 100, 300, False, False),
                                           (3, 7, 5, False, False)])
def test_gemm_skinny_epilogues(C, M, N, K, a_k, b_k):
    """Skinny kernels (one dimension <= 16): bias + ReLU + beta*C and the row-sum bias gradient."""
    torch.manual_seed(M * 7 + N + K)
    d = "cuda"
    A = torch.randn((M, K) if a_k else (K, M), device=d)
    B = torch.randn((N, K) if b_k else (K, N), device=d)
    ref = _ref_gemm(A, B, a_k, b_k)
    tol = 2e-4 * max(1.0, K ** 0.5)
    bias = torch.randn(N, device=d)
    out = torch.empty(M, N, device=d)
    C.gemm_f32(A, B, out, a_k, b_k, bias=bias, relu=True)
    _close(out, torch.relu(ref + bias), rtol=1e-4, atol=tol)
    prev = torch.randn(M, N, device=d)
    out = prev.clone()
    C.gemm_f32(A, B, out, a_k, b_k, beta=1.0)
    _close(out, ref + prev, rtol=1e-4, atol=tol)
    if not a_k:
        rs = torch.randn(M, device=d)
        rs0 = rs.clone()
        out = torch.empty(M, N, device=d)
        C.gemm_f32(A, B, out, a_k, b_k, rowsum=rs, rowsum_beta=1.0)
        _close(out, ref, rtol=1e-4, atol=tol)
        _close(rs, rs0 + A.double().sum(0).float(), rtol=1e-4, atol=1e-3)


def test_gather_batch_matches_index_select(C):
    """One-launch loader gather (samples + labels) == two index_selects, incl. F % 4 != 0."""
    from tutorial_torch_distributed_data_parallel_amd.data.synthetic import gather_batch

    torch.manual_seed(5)
    for shape in [(300, 9216), (50, 3, 7, 5), (9, 1)]:
        x = torch.randn(*shape, device="cuda")
        y = torch.randint(0, 10, (shape[0],), device="cuda")
        idx = torch.randint(0, shape[0], (37,), device="cuda")
        xb, yb = C.gather_batch(x, y, idx)
        assert xb.shape == (37,) + shape[1:]
        assert torch.equal(xb, x.index_select(0, idx)) and torch.equal(yb, y.index_select(0, idx))
        xb2, yb2 = gather_batch(x, y, idx[5:20])
        assert torch.equal(xb2, x[idx[5:20]]) and torch.equal(yb2, y[idx[5:20]])


@pytest.mark.parametrize("smoothing,reduction", [(0.0, "mean"), (0.1, "mean"), (0.0, "sum")])
def test_cross_entropy_fused_grad_matches_torch(smoothing, reduction):
    """Seeded with the cached unit seed (tdp.ops.backward) the logits gradient comes from the
    forward kernel (no backward launch); any other upstream gradient runs ce_bwd. Both vs torch."""
    import torch.nn.functional as F

    from tutorial_torch_distributed_data_parallel_amd import ops

    torch.manual_seed(3)
    x = torch.randn(128, 10, device="cuda") * 3
    y = torch.randint(0, 10, (128,), device="cuda")
    y[5] = -100  # ignored row
    ref_x = x.double().cpu().requires_grad_()
    ref = F.cross_entropy(ref_x, y.cpu(), ignore_index=-100, label_smoothing=smoothing,
                          reduction=reduction)
    ref.backward()
    for mode in ("seed", "scaled"):
        xi = x.clone().requires_grad_()
        loss = ops.cross_entropy(xi, y, label_smoothing=smoothing, reduction=reduction)
        if mode == "seed":
            ops.backward(loss)
            want = ref_x.grad
        else:
            (loss * 0.5).backward()
            want = ref_x.grad * 0.5
        torch.testing.assert_close(loss.double().cpu(), ref.detach(), rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(xi.grad.double().cpu(), want, rtol=1e-5, atol=1e-6)
