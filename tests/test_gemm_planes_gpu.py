"""Skinny GEMM from pre-split bf16 planes of A (csrc/gemm_planes.hip) against a float64 reference,
next to the split-bf16 fast GEMM it replaces on the toy-MLP's forward / input-gradient shapes.
The split itself must be exact (hi + mid + lo == x), and the GEMM must carry fp32 accuracy:
error / (|A| @ |B|) within the fp32 bound of tests/test_gemm_emu_gpu.py."""
import pytest
import torch

pytestmark = pytest.mark.gpu

U = 2.0 ** -24


@pytest.fixture(scope="module")
def C():
    from tutorial_torch_distributed_data_parallel_amd._native import native

    return native()


def _scaled_err(out, A, Bm):
    ref = A.double() @ Bm.double()
    scale = A.double().abs() @ Bm.double().abs()
    return ((out.double() - ref).abs() / scale.clamp_min(1e-30)).max().item()


def test_split_planes_exact(C):
    torch.manual_seed(0)
    x = torch.randn(37, 64, device="cuda") * torch.exp2(
        torch.randint(-30, 31, (37, 64), device="cuda").float())
    p = C.split_planes(x)
    assert p.dtype == torch.bfloat16 and p.shape == (3, 37, 64)
    s = p[0].double() + p[1].double() + p[2].double()
    assert torch.equal(s, x.double())
    # the head term is the RNE bf16 of x, the middle term that of the residual
    assert torch.equal(p[0], x.bfloat16())
    assert torch.equal(p[1], (x - p[0].float()).bfloat16())


SHAPES = [(128, 4096, 9216, True),   # toy-MLP fc1 forward
          (128, 4096, 4096, True),   # fc2 forward
          (128, 4096, 4096, False),  # fc2 input gradient (W stored [out][in])
          (130, 200, 64, True),      # ragged M / N edges
          (32, 128, 256, False),
          (300, 256, 512, True),     # several row tiles
          (1024, 512, 9216, True),   # tensor-sharded fc1 at W = 8 (the node's batch)
          (1024, 4096, 512, True)]   # its fc2 partial GEMM


@pytest.mark.parametrize("M,N,K,bk", SHAPES)
def test_planes_gemm_matches_fp64(C, M, N, K, bk):
    torch.manual_seed(M + 3 * N + 7 * K)
    A = torch.randn(M, K, device="cuda")
    B = torch.randn((N, K) if bk else (K, N), device="cuda")
    Bm = B.t() if bk else B
    out = torch.empty(M, N, device="cuda")
    C.gemm_planes(C.split_planes(A), B, out, bk)
    ref_fast = torch.empty(M, N, device="cuda")
    C.gemm_f32(A, B, ref_fast, True, bk)
    torch.cuda.synchronize()
    e = _scaled_err(out, A, Bm)
    e_fast = _scaled_err(ref_fast, A, Bm)
    bound = (8 + 2 * K ** 0.5) * U
    assert e < bound, (e, bound)
    assert e < 4 * e_fast + 16 * U, (e, e_fast)


@pytest.mark.parametrize("M,N,K,bk", SHAPES)
def test_planes_single_group_kernel_matches_fp64(C, M, N, K, bk):
    """The one-wave-group 3-stage variant (gemm_planes_set_cfg stages 3; the default, stages 4,
    sums each half of every K tile in its own wave group, so the two are not bitwise equal): the
    same fp32 bound, epilogues and split-K partials through the same paths."""
    torch.manual_seed(M + 3 * N + 7 * K)
    A = torch.randn(M, K, device="cuda")
    B = torch.randn((N, K) if bk else (K, N), device="cuda")
    Bm = B.t() if bk else B
    out = torch.empty(M, N, device="cuda")
    assert C.gemm_planes_set_cfg(3, 0, 0)
    try:
        C.gemm_planes(C.split_planes(A), B, out, bk)
        b = torch.randn(N, device="cuda")
        y = torch.empty(M, N, device="cuda")
        C.gemm_planes(C.split_planes(A), B, y, bk, bias=b, relu=True)
        torch.cuda.synchronize()
    finally:
        C.gemm_planes_set_cfg(4, 0, 0)
    e = _scaled_err(out, A, Bm)
    assert e < (8 + 2 * K ** 0.5) * U, e
    ref = torch.relu(A.double() @ Bm.double() + b.double())
    torch.testing.assert_close(y.double(), ref, rtol=1e-4, atol=1e-4 * K ** 0.5)


def test_planes_gemm_epilogues_and_out_planes(C):
    torch.manual_seed(1)
    M, N, K = 128, 512, 1024
    A = torch.randn(M, K, device="cuda")
    W = torch.randn(N, K, device="cuda") / 32
    b = torch.randn(N, device="cuda")
    gate = torch.randn(M, N, device="cuda")
    y = torch.empty(M, N, device="cuda")
    op = torch.empty(3, M, N, device="cuda", dtype=torch.bfloat16)
    C.gemm_planes(C.split_planes(A), W, y, True, bias=b, relu=True, gate=gate, out_planes=op)
    ref = torch.relu(A.double() @ W.double().t() + b.double()) * (gate > 0).double()
    torch.testing.assert_close(y.double(), ref, rtol=1e-5, atol=1e-5)
    assert torch.equal(op, C.split_planes(y))
    # single split (no workspace): the in-kernel epilogue path
    A2 = torch.randn(256, 128, device="cuda")
    W2 = torch.randn(1024, 128, device="cuda")
    b2 = torch.randn(1024, device="cuda")
    y2 = torch.empty(256, 1024, device="cuda")
    op2 = torch.empty(3, 256, 1024, device="cuda", dtype=torch.bfloat16)
    assert C.gemm_planes_plan(256, 1024, 128, 256)[0] == 1
    C.gemm_planes(C.split_planes(A2), W2, y2, True, bias=b2, relu=True, out_planes=op2)
    ref2 = torch.relu(A2.double() @ W2.double().t() + b2.double())
    torch.testing.assert_close(y2.double(), ref2, rtol=1e-5, atol=1e-5)
    assert torch.equal(op2, C.split_planes(y2))


def test_planes_gemm_rejects_bad_shapes(C):
    A = torch.randn(16, 48, device="cuda")  # K % 32 != 0
    with pytest.raises(RuntimeError):
        C.gemm_planes(C.split_planes(A), torch.randn(64, 48, device="cuda"),
                      torch.empty(16, 64, device="cuda"), True)


def test_gather_batch_emits_planes(C):
    torch.manual_seed(2)
    x = torch.randn(64, 512, device="cuda")
    y = torch.randint(0, 10, (64,), device="cuda")
    idx = torch.randint(0, 64, (32,), device="cuda")
    xb, yb, p = C.gather_batch(x, y, idx, planes=True)
    assert torch.equal(xb, x[idx]) and torch.equal(yb, y[idx])
    assert torch.equal(p, C.split_planes(x[idx]))


def test_mlp_linear_chain_planes_vs_split_path():
    """fc1 -> fc2 -> fc3 of the toy MLP shape family (smaller widths) through ops.linear with the
    planes path on and off: the forward / gradients agree to fp32 accuracy and both match fp64."""
    from tutorial_torch_distributed_data_parallel_amd import ops
    from tutorial_torch_distributed_data_parallel_amd.data.synthetic import gather_batch
    import importlib

    L = importlib.import_module("tutorial_torch_distributed_data_parallel_amd.ops.linear")

    torch.manual_seed(3)
    data = torch.randn(256, 1024, device="cuda")
    lab = torch.randint(0, 10, (256,), device="cuda")
    idx = torch.randperm(256, device="cuda")[:128]
    ws = [torch.randn(1024, 1024, device="cuda") / 32, torch.randn(512, 1024, device="cuda") / 32,
          torch.randn(10, 512, device="cuda") / 22]
    bs = [torch.randn(w.shape[0], device="cuda") / 10 for w in ws]
    res = {}
    for on in (True, False):
        old = L.set_planes(on)
        try:
            x, _ = gather_batch(data, lab, idx)
            assert (getattr(x, "_tdp_planes", None) is not None) == on
            p = [t.clone().requires_grad_() for t in ws + bs]
            h = ops.linear(x.reshape(128, -1), p[0], p[3], relu=True)
            h = ops.linear(h, p[1], p[4], relu=True)
            out = ops.linear(h, p[2], p[5])
            out.backward(torch.linspace(-1, 1, out.numel(), device="cuda").view_as(out))
            torch.cuda.synchronize()
            res[on] = [out.detach()] + [t.grad for t in p]
        finally:
            L.set_planes(old)
    xd = data[idx].double()
    pd = [t.double().requires_grad_() for t in ws + bs]
    h = torch.relu(xd @ pd[0].t() + pd[3])
    h = torch.relu(h @ pd[1].t() + pd[4])
    out = h @ pd[2].t() + pd[5]
    out.backward(torch.linspace(-1, 1, out.numel(), device="cuda", dtype=torch.float64)
                 .view_as(out))
    ref = [out.detach()] + [t.grad for t in pd]
    for a, b, r in zip(res[True], res[False], ref):
        torch.testing.assert_close(a.double(), r, rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("O,I,B", [(10, 1024, 128), (3, 1024, 128), (16, 1024, 128),
                                   (10, 4100, 128), (10, 4096, 100), (9, 68, 37)])
def test_head_bwd_one_launch(C, O, I, B):
    """fc3-style head backward (csrc/gemm_skinny.hip head_bwd): dx = g W gated, its planes,
    dW = g^T x and db = sum g, against fp64 (ragged column / batch-slice edges included)."""
    torch.manual_seed(O + I + B)
    g = torch.randn(B, O, device="cuda")
    x = torch.relu(torch.randn(B, I, device="cuda"))
    w = torch.randn(O, I, device="cuda")
    dx = torch.empty(B, I, device="cuda")
    dw = torch.empty(O, I, device="cuda")
    db = torch.empty(O, device="cuda")
    ok, pl = C.head_bwd(g, x, w, dx, dw, db=db, gate=x, planes=True)
    torch.cuda.synchronize()
    assert ok
    ref_dx = (g.double() @ w.double()) * (x > 0).double()
    torch.testing.assert_close(dx.double(), ref_dx, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(dw.double(), g.double().t() @ x.double(), rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(db.double(), g.double().sum(0), rtol=1e-5, atol=1e-5)
    assert torch.equal(pl, C.split_planes(dx))


def test_cursor_gather_walks_the_epoch_order():
    """EpochCursor: each gather reads the next batch of the installed order and advances the
    device-side position itself (also inside a captured graph); set_order rewinds."""
    from tutorial_torch_distributed_data_parallel_amd.data.synthetic import (
        EpochCursor, gather_batch_cursor)

    torch.manual_seed(5)
    x = torch.randn(512, 256, device="cuda")
    y = torch.randint(0, 10, (512,), device="cuda")
    order = torch.randperm(512, device="cuda")
    assert EpochCursor.fits(x, y, 64)
    cur = EpochCursor(512, 64, "cuda")
    cur.set_order(order)
    for k in range(3):
        xb, yb = gather_batch_cursor(x, y, cur)
        sl = order[64 * k: 64 * (k + 1)]
        assert torch.equal(xb, x[sl]) and torch.equal(yb, y[sl])
    assert int(cur.state[0]) == 192 and int(cur.state[1]) == 0
    # captured: replays advance too
    static = {}

    def step():
        static["xb"], static["yb"] = gather_batch_cursor(x, y, cur)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()  # warm-up (advances to 256)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    cur.set_order(order)
    for k in range(2):
        g.replay()
        torch.cuda.synchronize()
        sl = order[64 * k: 64 * (k + 1)]
        assert torch.equal(static["xb"], x[sl]) and torch.equal(static["yb"], y[sl])


def test_cursor_gather_sliced_rows_and_legacy_state(C):
    """Wide rows: several workgroups per row count on per-row counters (state [2 + batch]), one
    arrival per row on the shared counter; all counters re-armed. A [2] state (no per-row
    counters) still works with one workgroup per row. Captured replays advance both ways."""
    from tutorial_torch_distributed_data_parallel_amd.data.synthetic import (
        EpochCursor, gather_batch_cursor)

    torch.manual_seed(6)
    x = torch.randn(300, 4096, device="cuda")
    y = torch.randint(0, 10, (300,), device="cuda")
    order = torch.randperm(300, device="cuda")
    cur = EpochCursor(300, 32, "cuda")
    assert cur.state.numel() == 34
    cur.set_order(order)
    for k in range(4):
        xb, yb = gather_batch_cursor(x, y, cur)
        sl = order[32 * k: 32 * (k + 1)]
        assert torch.equal(xb, x[sl]) and torch.equal(yb, y[sl])
    assert int(cur.state[0]) == 128 and int(cur.state[1:].abs().sum()) == 0
    legacy = torch.zeros(2, dtype=torch.long, device="cuda")
    for k in range(2):
        xb, yb, p = C.gather_batch(x, y, order, planes=True, cursor=legacy, batch=32)
        sl = order[32 * k: 32 * (k + 1)]
        assert torch.equal(xb, x[sl]) and torch.equal(yb, y[sl])
        assert torch.equal(p[0].double() + p[1].double() + p[2].double(), xb.double())
    assert int(legacy[0]) == 64 and int(legacy[1]) == 0
    static = {}

    def step():
        static["xb"], static["yb"] = gather_batch_cursor(x, y, cur)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    cur.set_order(order)
    for k in range(3):
        g.replay()
        torch.cuda.synchronize()
        sl = order[32 * k: 32 * (k + 1)]
        assert torch.equal(static["xb"], x[sl]) and torch.equal(static["yb"], y[sl])
    assert int(cur.state[0]) == 96 and int(cur.state[1:].abs().sum()) == 0


@pytest.mark.parametrize("local1d", [True, False])
def test_batchnorm1d_planes_and_local_merge_match_torch(local1d):
    """Linear -> BatchNorm1d(+ReLU) -> Linear (the toy MLP's SyncBN config at one rank): the BN
    forward merges its own statistics (one launch) and emits bf16 planes for the next skinny GEMM,
    its backward emits the input gradient's planes; forward, gradients and running statistics
    match torch in fp64 -- with the one-launch whole-column kernels (local1d) and without."""
    import torch.nn.functional as F

    from tutorial_torch_distributed_data_parallel_amd import ops
    from tutorial_torch_distributed_data_parallel_amd.ops import norm as norm_mod

    prev = norm_mod.set_local1d(local1d)
    try:
        _bn1d_chain(F, ops)
    finally:
        norm_mod.set_local1d(prev)


def _bn1d_chain(F, ops):

    torch.manual_seed(11)
    B, I, H, O = 128, 512, 1024, 1024
    x = torch.randn(B, I, device="cuda")
    w1 = (torch.randn(H, I, device="cuda") / 22).requires_grad_()
    b1 = torch.randn(H, device="cuda").requires_grad_()
    g = (torch.rand(H, device="cuda") + 0.5).requires_grad_()
    bb = (torch.randn(H, device="cuda") * 0.1).requires_grad_()
    w2 = (torch.randn(O, H, device="cuda") / 32).requires_grad_()
    rm, rv = torch.zeros(H, device="cuda"), torch.ones(H, device="cuda")
    nbt = torch.zeros((), dtype=torch.long, device="cuda")
    h = ops.linear(x, w1, b1)
    a = ops.batch_norm(h, rm, rv, g, bb, training=True, momentum=0.1, eps=1e-5, relu=True,
                       num_batches_tracked=nbt)
    assert getattr(a, "_tdp_planes", None) is not None
    out = ops.linear(a, w2)
    seed = torch.linspace(-1, 1, out.numel(), device="cuda").view_as(out)
    out.backward(seed)
    torch.cuda.synchronize()
    prm = [t.detach().double().requires_grad_() for t in (w1, b1, g, bb, w2)]
    rm2, rv2 = torch.zeros(H, dtype=torch.float64, device="cuda"), \
        torch.ones(H, dtype=torch.float64, device="cuda")
    hr = x.double() @ prm[0].t() + prm[1]
    ar = torch.relu(F.batch_norm(hr, rm2, rv2, prm[2], prm[3], training=True, momentum=0.1,
                                 eps=1e-5))
    outr = ar @ prm[4].t()
    outr.backward(seed.double())
    torch.testing.assert_close(out.double(), outr, rtol=1e-4, atol=1e-4)
    for t, r in zip((w1, b1, g, bb, w2), prm):
        torch.testing.assert_close(t.grad.double(), r.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(rm.double(), rm2, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rv.double(), rv2, rtol=1e-5, atol=1e-6)
    assert int(nbt) == 1


def test_split_k_reduce_is_deterministic(C):
    """The split-K planes GEMM sums its partials in split order in one reduce launch: repeated
    launches give bitwise-identical outputs and output planes (shapes of the toy MLP's fc1 /
    fc2 forward and a ragged one)."""
    torch.manual_seed(5)
    for (M, N, K, bk) in [(128, 4096, 9216, True), (128, 4096, 4096, False), (300, 256, 512, True)]:
        A = torch.randn(M, K, device="cuda")
        B = torch.randn((N, K) if bk else (K, N), device="cuda")
        bias = torch.randn(N, device="cuda")
        outs = []
        for _ in range(3):
            out = torch.empty(M, N, device="cuda")
            op = torch.empty((3, M, N), dtype=torch.bfloat16, device="cuda")
            C.gemm_planes(C.split_planes(A), B, out, bk, bias=bias, relu=True, out_planes=op)
            outs.append((out, op))
        for out, op in outs[1:]:
            assert torch.equal(out, outs[0][0]) and torch.equal(op, outs[0][1])
        ref = torch.relu((A.double() @ (B.double().t() if bk else B.double())) + bias.double())
        # |C| ~ sqrt(K): fp32 accumulation over K terms, scaled like the other planes tests
        torch.testing.assert_close(outs[0][0].double(), ref, rtol=1e-4, atol=2e-5 * K ** 0.5)


@pytest.mark.parametrize("N,Cn", [(128, 4096), (37, 16), (64, 48), (300, 1024), (512, 2064),
                                  (2, 32)])
@pytest.mark.parametrize("relu,affine", [(True, True), (False, False)])
def test_bn1d_local_kernels_match_the_split_path(N, Cn, relu, affine):
    """csrc/norm.hip bn1d_local_fwd / bn1d_local_bwd (a workgroup per 16 channels over all rows)
    against the split kernels they replace (bn_moments + bn_elemt_local; bn_bwd_reduce +
    bn_bwd_elemt) and an fp64 torch oracle: y, stats, running statistics, mask, planes, dx,
    dw, db."""
    from tutorial_torch_distributed_data_parallel_amd._native import native

    C = native()
    torch.manual_seed(N + Cn)
    x = torch.randn(N, Cn, device="cuda") * 1.7 + 0.4
    w = torch.randn(Cn, device="cuda") if affine else None
    b = torch.randn(Cn, device="cuda") if affine else None
    rm1, rv1 = torch.randn(Cn, device="cuda"), torch.rand(Cn, device="cuda") + 0.5
    rm2, rv2 = rm1.clone(), rv1.clone()
    nb1, nb2 = (torch.zeros(1, dtype=torch.long, device="cuda") for _ in range(2))
    mk1 = torch.empty((N, Cn // 4), dtype=torch.uint8, device="cuda") if relu else None
    mk2 = torch.empty((N, Cn // 4), dtype=torch.uint8, device="cuda") if relu else None
    pl1, pl2 = (torch.empty((3, N, Cn), dtype=torch.bfloat16, device="cuda") for _ in range(2))
    y1, st1 = C.bn1d_local_fwd(x, w, b, relu, 1e-5, 0.1, rmean=rm1, rvar=rv1, num_batches=nb1,
                               mask_out=mk1, planes_out=pl1)
    mom = C.bn_moments(x)[0]
    y2, st2 = C.bn_elemt_local(x, mom, w, b, relu, 1e-5, 0.1, rmean=rm2, rvar=rv2,
                               num_batches=nb2, mask_out=mk2, planes_out=pl2)
    torch.testing.assert_close(st1, st2, rtol=2e-5, atol=2e-5)
    torch.testing.assert_close(y1, y2, rtol=2e-5, atol=2e-5)
    torch.testing.assert_close(rm1, rm2, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rv1, rv2, rtol=1e-5, atol=1e-6)
    assert int(nb1) == 1 == int(nb2)
    xd = x.double()
    yr = torch.nn.functional.batch_norm(xd, None, None, None if w is None else w.double(),
                                        None if b is None else b.double(), True, 0.0, 1e-5)
    if relu:
        yr = torch.relu(yr)
        bits = (y1 > 0).view(N, Cn // 4, 4).to(torch.int32)
        packed = (bits * torch.tensor([1, 2, 4, 8], device="cuda", dtype=torch.int32)).sum(-1)
        assert torch.equal(mk1.to(torch.int32), packed)
    torch.testing.assert_close(y1.double(), yr, rtol=1e-4, atol=1e-4)
    # the planes are the exact split of y
    assert torch.equal(pl1.double().sum(0).float(), y1)
    dy = torch.randn(N, Cn, device="cuda")
    dw1, db1, dw2, db2 = (torch.empty(Cn, device="cuda") for _ in range(4))
    dpl = torch.empty((3, N, Cn), dtype=torch.bfloat16, device="cuda")
    dx1 = C.bn1d_local_bwd(dy, x, st1, w, mask=mk1, dw=dw1 if affine else None,
                           db=db1 if affine else None, planes_out=dpl)
    kw = {} if mk2 is None else {"mask": mk2}
    sums = C.bn_bwd_reduce(dy, x, st2, None, dw2 if affine else None, db2 if affine else None,
                           0.0, **kw)
    dx2 = C.bn_bwd_elemt(dy, x, st2, w, sums, None, False, **kw)[0]
    torch.testing.assert_close(dx1, dx2, rtol=1e-4, atol=1e-4)
    if affine:
        torch.testing.assert_close(dw1, dw2, rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(db1, db2, rtol=1e-4, atol=1e-4)
    # fp64 oracle of the input gradient
    xr = xd.clone().requires_grad_()
    out = torch.nn.functional.batch_norm(xr, None, None, None if w is None else w.double(),
                                         None if b is None else b.double(), True, 0.0, 1e-5)
    if relu:
        out = torch.relu(out)
    (out * dy.double()).sum().backward()
    torch.testing.assert_close(dx1.double(), xr.grad, rtol=1e-3, atol=1e-3)



@pytest.mark.parametrize("Cn", [16, 1024])
def test_bn1d_sync_halves_match_the_split_path(Cn):
    """SyncBatchNorm halves of the whole-column kernels: bn1d_moments (= bn_moments), then --
    over the all-gathered moments of three ranks (one of them empty, dropped as torch does) --
    bn1d_gathered_fwd (= bn_merge + bn_elemt, bitwise: the same merge order and formulas), and
    bn1d_sums (= bn_bwd_reduce: local sums, dw, db)."""
    from tutorial_torch_distributed_data_parallel_amd._native import native

    C = native()
    torch.manual_seed(Cn)
    xs = [torch.randn(n, Cn, device="cuda") * (1 + r) + r for r, n in enumerate((128, 77, 200))]
    moms = [C.bn1d_moments(x) for x in xs]
    for x, m in zip(xs, moms):
        ref = C.bn_moments(x)[0]
        torch.testing.assert_close(m[:2 * Cn], ref[:2 * Cn], rtol=1e-5, atol=1e-5)
        assert m[2 * Cn].item() == x.shape[0]
    empty = torch.zeros(2 * Cn + 1, device="cuda")  # a rank with no samples
    gathered = torch.cat([moms[0], empty, moms[1], moms[2]])
    x = xs[1]
    w, b = torch.randn(Cn, device="cuda"), torch.randn(Cn, device="cuda")
    rm1, rv1 = torch.randn(Cn, device="cuda"), torch.rand(Cn, device="cuda") + 0.5
    rm2, rv2 = rm1.clone(), rv1.clone()
    nb1, nb2 = (torch.zeros(1, dtype=torch.long, device="cuda") for _ in range(2))
    mk1, mk2 = (torch.empty((x.shape[0], Cn // 4), dtype=torch.uint8, device="cuda")
                for _ in range(2))
    y1, st1 = C.bn1d_gathered_fwd(x, gathered, w, b, True, 1e-5, 0.1, rmean=rm1, rvar=rv1,
                                  num_batches=nb1, mask_out=mk1)
    st2 = C.bn_merge(gathered, Cn, 1e-5, 0.1, rm2, rv2, nb2)
    y2 = C.bn_elemt(x, st2, w, b, True, None, mask_out=mk2)
    assert torch.equal(st1, st2) and torch.equal(y1, y2) and torch.equal(mk1, mk2)
    assert torch.equal(rm1, rm2) and torch.equal(rv1, rv2) and int(nb1) == int(nb2) == 1
    xa = torch.cat(xs).double()
    torch.testing.assert_close(st1[:Cn].double(), xa.mean(0), rtol=1e-5, atol=1e-5)
    dy = torch.randn_like(x)
    dw1, db1, dw2, db2 = (torch.empty(Cn, device="cuda") for _ in range(4))
    s1 = C.bn1d_sums(dy, x, st1, mask=mk1, dw=dw1, db=db1)
    s2 = C.bn_bwd_reduce(dy, x, st2, None, dw2, db2, 0.0, mask=mk2)
    torch.testing.assert_close(s1, s2, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dw1, dw2, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(db1, db2, rtol=1e-4, atol=1e-4)
