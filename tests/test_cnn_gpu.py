"""Conv / pooling / dropout / residual kernels and the CNN models vs a float64 PyTorch reference."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CONVS = [
    # N, C, H, W, Cout, R, stride, pad
    (2, 3, 63, 63, 64, 11, 4, 2),     # AlexNet conv1 (scaled input)
    (2, 64, 15, 15, 192, 5, 1, 2),    # AlexNet conv2
    (2, 192, 13, 13, 384, 3, 1, 1),   # AlexNet conv3
    (3, 64, 14, 14, 256, 1, 1, 0),    # ResNet 1x1 expand
    (2, 256, 14, 14, 512, 1, 2, 0),   # ResNet downsample projection
    (2, 128, 15, 15, 128, 3, 2, 1),   # ResNet v1.5 strided 3x3
    (2, 3, 40, 40, 64, 7, 2, 3),      # ResNet stem
    (1, 5, 9, 11, 7, 3, 1, 1),        # odd everything
    (2, 7, 10, 9, 33, 2, 3, 0),       # stride > kernel
]


def _ref(x, w, b, s, p, relu):
    y = F.conv2d(x.double().cpu(), w.double().cpu(), None if b is None else b.double().cpu(),
                 s, p)
    return F.relu(y) if relu else y


@pytest.fixture(params=["nhwc", "nchw"])
def conv_path(request):
    from tutorial_torch_distributed_data_parallel_amd.ops import conv as conv_mod

    conv_mod.FORCE_NCHW = request.param == "nchw"
    yield request.param
    conv_mod.FORCE_NCHW = False


@pytest.mark.parametrize("N,C,H,W,Co,R,s,p", CONVS)
@pytest.mark.parametrize("relu", [False, True])
def test_conv2d_fwd_bwd(N, C, H, W, Co, R, s, p, relu, conv_path):
    from tutorial_torch_distributed_data_parallel_amd import ops

    torch.manual_seed(N * 1000 + C * 10 + R)
    x = torch.randn(N, C, H, W, device="cuda", requires_grad=True)
    w = (torch.randn(Co, C, R, R, device="cuda") / (C * R * R) ** 0.5).requires_grad_()
    b = torch.randn(Co, device="cuda", requires_grad=True)
    y = ops.conv2d(x, w, b, s, p, relu=relu)
    xr = x.detach().double().cpu().requires_grad_()
    wr = w.detach().double().cpu().requires_grad_()
    br = b.detach().double().cpu().requires_grad_()
    yr = F.conv2d(xr, wr, br, s, p)
    if relu:
        yr = F.relu(yr)
    torch.testing.assert_close(y.double().cpu(), yr, rtol=1e-4, atol=1e-4)
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy.double().cpu())
    K = Co * R * R
    torch.testing.assert_close(x.grad.double().cpu(), xr.grad, rtol=1e-4,
                               atol=2e-4 * max(1.0, K ** 0.5))
    P = N * y.shape[2] * y.shape[3]
    torch.testing.assert_close(w.grad.double().cpu(), wr.grad, rtol=1e-4,
                               atol=2e-4 * max(1.0, P ** 0.5))
    torch.testing.assert_close(b.grad.double().cpu(), br.grad, rtol=1e-4,
                               atol=2e-4 * max(1.0, P ** 0.5))


def test_conv2d_nhwc_layouts():
    """channels_last in -> channels_last out; NCHW inputs are accepted and converted."""
    from tutorial_torch_distributed_data_parallel_amd import ops

    torch.manual_seed(5)
    w = torch.randn(32, 16, 3, 3, device="cuda")
    for fmt in (torch.contiguous_format, torch.channels_last):
        x = torch.randn(2, 16, 9, 9, device="cuda").contiguous(memory_format=fmt)
        y = ops.conv2d(x, w, None, 1, 1)
        assert y.is_contiguous(memory_format=torch.channels_last)
        torch.testing.assert_close(y.double().cpu(),
                                   F.conv2d(x.double().cpu(), w.double().cpu(), None, 1, 1),
                                   rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("shape", [(4, 64, 14, 14), (8, 256, 7, 7), (2, 3, 5, 5)])
def test_batchnorm_channels_last(shape):
    """BatchNorm2d on NHWC activations runs the [pixels, C] kernels; compare with torch."""
    from tutorial_torch_distributed_data_parallel_amd import nn as tnn

    torch.manual_seed(1)
    bn = tnn.BatchNorm2d(shape[1], relu=True).cuda()
    ref = torch.nn.BatchNorm2d(shape[1]).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        ref.weight.copy_(bn.weight)
        ref.bias.copy_(bn.bias)
    x = (torch.randn(shape, device="cuda") * 2 + 0.5).contiguous(memory_format=torch.channels_last)
    x.requires_grad_()
    xr = x.detach().clone().requires_grad_()
    y = bn(x)
    yr = torch.relu(ref(xr))
    assert y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y, yr, rtol=1e-4, atol=1e-4)
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy)
    torch.testing.assert_close(x.grad, xr.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(bn.weight.grad, ref.weight.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(bn.running_var, ref.running_var, rtol=1e-5, atol=1e-5)
    bn.eval()
    ref.eval()
    torch.testing.assert_close(bn(x.detach()), torch.relu(ref(x.detach())), rtol=1e-4, atol=1e-4)


def test_conv2d_no_bias_wgrad_only():
    from tutorial_torch_distributed_data_parallel_amd import ops

    torch.manual_seed(3)
    x = torch.randn(4, 64, 28, 28, device="cuda")
    w = torch.randn(128, 64, 3, 3, device="cuda", requires_grad=True)
    y = ops.conv2d(x, w, None, 1, 1)
    y.sum().backward()
    wr = w.detach().double().cpu().requires_grad_()
    F.conv2d(x.double().cpu(), wr, None, 1, 1).sum().backward()
    torch.testing.assert_close(w.grad.double().cpu(), wr.grad, rtol=1e-4, atol=5e-2)


FMTS = [torch.contiguous_format, torch.channels_last]


@pytest.mark.parametrize("fmt", FMTS)
@pytest.mark.parametrize("k,s,p,H", [(3, 2, 0, 55), (3, 2, 0, 13), (3, 2, 1, 112), (2, 2, 0, 8)])
@pytest.mark.parametrize("C", [5, 64])  # 64: the 4-channel vector kernels (channels_last)
def test_maxpool(k, s, p, H, fmt, C):
    from tutorial_torch_distributed_data_parallel_amd import ops

    torch.manual_seed(H)
    x = torch.randn(2, C, H, H + 1, device="cuda").contiguous(memory_format=fmt)
    x.requires_grad_()
    y = ops.max_pool2d(x, k, s, p)
    xr = x.detach().clone().requires_grad_()
    yr = F.max_pool2d(xr, k, s, p)
    torch.testing.assert_close(y, yr, rtol=0, atol=0)
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy)
    torch.testing.assert_close(x.grad, xr.grad, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("fmt", FMTS)
@pytest.mark.parametrize("H,W,P,Q", [(13, 13, 6, 6), (7, 7, 1, 1), (10, 7, 3, 4), (5, 5, 6, 6)])
def test_adaptive_avgpool(H, W, P, Q, fmt):
    from tutorial_torch_distributed_data_parallel_amd import ops

    x = torch.randn(2, 3, H, W, device="cuda").contiguous(memory_format=fmt)
    x.requires_grad_()
    y = ops.adaptive_avg_pool2d(x, (P, Q))
    xr = x.detach().clone().requires_grad_()
    yr = F.adaptive_avg_pool2d(xr, (P, Q))
    torch.testing.assert_close(y, yr, rtol=1e-5, atol=1e-6)
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy)
    torch.testing.assert_close(x.grad, xr.grad, rtol=1e-5, atol=1e-6)


def test_dropout_statistics_and_backward():
    from tutorial_torch_distributed_data_parallel_amd import ops

    torch.manual_seed(0)
    x = torch.ones(1 << 20, device="cuda", requires_grad=True)
    y = ops.dropout(x, 0.5, True)
    kept = (y != 0)
    frac = kept.float().mean().item()
    assert abs(frac - 0.5) < 0.005
    torch.testing.assert_close(y[kept], torch.full_like(y[kept], 2.0))
    y.backward(torch.ones_like(y))
    torch.testing.assert_close(x.grad, y.detach())  # same mask and scale
    y2 = ops.dropout(x, 0.5, True)
    assert not torch.equal(y2, y)  # fresh seed per call
    assert ops.dropout(x, 0.5, False) is x


@pytest.mark.parametrize("fmt", FMTS)
def test_add_relu(fmt):
    from tutorial_torch_distributed_data_parallel_amd import ops

    a = torch.randn(3, 8, 5, 5, device="cuda").contiguous(memory_format=fmt).requires_grad_()
    b = torch.randn(3, 8, 5, 5, device="cuda").requires_grad_()  # NCHW: converted to a's layout
    y = ops.add_relu(a, b)
    torch.testing.assert_close(y, F.relu(a + b))
    dy = torch.randn_like(y)
    y.backward(dy)
    ref = dy * ((a + b) > 0)
    torch.testing.assert_close(a.grad, ref)
    torch.testing.assert_close(b.grad, ref)


@pytest.mark.parametrize("name,hw,n", [("alexnet", 224, 2), ("resnet50", 64, 8)])
def test_model_matches_cpu_reference(name, hw, n):
    """Whole model on GPU (native fp32 kernels) vs the same weights in float64 on CPU (ATen).

    Gradients are compared in eval mode: train-mode batch norm over ResNet's 2x2 layer4 maps
    (32 values per channel here) is so ill-conditioned that even CPU fp32 differs from fp64 by
    ~25% in layer4's weight gradients; the train-mode forward is still compared."""
    from tutorial_torch_distributed_data_parallel_amd.models.registry import build_model

    torch.manual_seed(0)
    m_cpu = build_model(name).double()
    m_gpu = build_model(name)
    m_gpu.load_state_dict(m_cpu.state_dict())
    m_gpu.cuda()
    x = torch.randn(n, 3, hw, hw, dtype=torch.float64)
    if name == "resnet50":
        with torch.no_grad():
            y_cpu = m_cpu.train()(x)
            y_gpu = m_gpu.train()(x.float().cuda())
        torch.testing.assert_close(y_gpu.double().cpu(), y_cpu, rtol=2e-3, atol=2e-3)
        torch.testing.assert_close(m_gpu.bn1.running_var.double().cpu(), m_cpu.bn1.running_var,
                                   rtol=1e-4, atol=1e-5)
    m_cpu.eval()
    m_gpu.eval()
    y_cpu = m_cpu(x)
    y_gpu = m_gpu(x.float().cuda())
    torch.testing.assert_close(y_gpu.double().cpu(), y_cpu, rtol=2e-3, atol=2e-3)
    y_cpu.square().sum().backward()
    y_gpu.square().sum().backward()
    # relative L2 error per parameter: a ReLU whose pre-activation rounds to the other side of 0
    # in fp32 vs fp64 (it happens ~1 in 1e5 elements) legitimately flips single gradient entries.
    # Noise floor: stock ATen fp32 on the CPU vs this fp64 reference gives 3.6e-3 on ResNet-50's
    # conv1.weight (2.6e-3 on layer2.2.conv3.weight) for this very input -- the bound sits above it.
    worst = []
    for (pn, pc), (_, pg) in zip(m_cpu.named_parameters(), m_gpu.named_parameters()):
        err = (pg.grad.double().cpu() - pc.grad).norm().item() / (pc.grad.norm().item() + 1e-12)
        worst.append((err, pn))
    worst.sort(reverse=True)
    assert worst[0][0] <= 5e-3, worst[:5]


@pytest.mark.parametrize("orient", [-1, 0, 1])
@pytest.mark.parametrize("override", [(0, 0, 0), (2, 0, 0), (1, 32, 0), (2, 8, 2), (1, 3, 3)])
@pytest.mark.parametrize("Co,C,R", [(192, 64, 5), (256, 128, 3)])
def test_conv_wgrad_plans(orient, override, Co, C, R):
    """Every weight-gradient plan (dW / dW^T orientation, tile width, split-K, pipeline depth)
    the planner can pick matches the float64 reference."""
    from tutorial_torch_distributed_data_parallel_amd import ops
    from tutorial_torch_distributed_data_parallel_amd._native import native

    N_ = native()
    torch.manual_seed(Co + C + R)
    x = torch.randn(4, C, 13, 13, device="cuda").contiguous(memory_format=torch.channels_last)
    x.requires_grad_()
    w = (torch.randn(Co, C, R, R, device="cuda") / (C * R * R) ** 0.5).requires_grad_()
    dy = torch.randn(4, Co, 13, 13, device="cuda")
    try:
        N_.conv_set_wgrad_transposed(orient)
        N_.gemm_f32_set_override(*override)
        y = ops.conv2d(x, w, None, 1, R // 2)
        y.backward(dy)
        torch.cuda.synchronize()
    finally:
        N_.conv_set_wgrad_transposed(-1)
        N_.gemm_f32_set_override(0, 0, 0)
    xr = x.detach().double().cpu().requires_grad_()
    wr = w.detach().double().cpu().requires_grad_()
    yr = F.conv2d(xr, wr, None, 1, R // 2)
    yr.backward(dy.double().cpu())
    torch.testing.assert_close(y.double().cpu(), yr, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(x.grad.double().cpu(), xr.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(w.grad.double().cpu(), wr.grad, rtol=1e-4, atol=2e-3)


@pytest.mark.parametrize("downsample", [False, True, "stride1"])
def test_bottleneck_fused_join_matches_unfused(downsample):
    """relu(bn3(conv3) + identity) fused into bn3's normalisation (and its backward writing the
    identity gradient) == separate bn3 + add_relu; the block input's two gradients meet in one
    shared buffer (conv1's input-gradient GEMM with beta = 1, the strided downsample phase with
    copy4d accumulate); running stats and num_batches_tracked are updated on the device."""
    import copy

    from tutorial_torch_distributed_data_parallel_amd.models.resnet import Bottleneck
    from tutorial_torch_distributed_data_parallel_amd.nn import BatchNorm2d, Conv2d

    torch.manual_seed(0)
    inp, planes, stride = {False: (128, 32, 1), True: (64, 32, 2),
                           "stride1": (64, 32, 1)}[downsample]
    ds = torch.nn.Sequential(Conv2d(inp, planes * 4, 1, stride=stride, bias=False),
                             BatchNorm2d(planes * 4)) if downsample else None
    a = Bottleneck(inp, planes, stride, ds).cuda()
    b = copy.deepcopy(a)
    b._fused_join = False
    x = torch.randn(8, inp, 28, 28, device="cuda").contiguous(memory_format=torch.channels_last)
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ya, yb = a(xa), b(xb)
    torch.testing.assert_close(ya, yb, atol=1e-5, rtol=1e-5)
    g = torch.randn_like(ya)
    ya.backward(g)
    yb.backward(g)
    torch.testing.assert_close(xa.grad, xb.grad, atol=1e-4, rtol=1e-4)
    for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
        torch.testing.assert_close(p.grad, q.grad, atol=1e-4, rtol=1e-4, msg=lambda m: f"{n}: {m}")
    for (n, p), (_, q) in zip(a.named_buffers(), b.named_buffers()):
        torch.testing.assert_close(p, q, atol=1e-6, rtol=1e-5, msg=lambda m: f"{n}: {m}")
    assert int(a.bn3.num_batches_tracked) == 1


@pytest.mark.parametrize("case", ["pad_nchw", "rows_phase", "zero", "transpose", "acc_rows",
                                  "acc_generic", "acc_zero"])
def test_copy4d(case):
    """csrc/elementwise.hip copy4d: strided copy over dst's shape, zeros outside src;
    accumulate: dst += src where src has the index."""
    from tutorial_torch_distributed_data_parallel_amd._native import native

    C = native()
    g = torch.Generator(device="cuda").manual_seed(0)
    if case == "pad_nchw":
        src = torch.randn(4, 3, 9, 7, device="cuda", generator=g)
        dst = torch.empty(4, 4, 9, 7, device="cuda").contiguous(memory_format=torch.channels_last)
        ref = torch.cat([src, torch.zeros(4, 1, 9, 7, device="cuda")], 1)
    elif case == "rows_phase":
        src = torch.randn(2, 8, 5, 6, device="cuda", generator=g).contiguous(
            memory_format=torch.channels_last)
        big = torch.zeros(2, 8, 10, 12, device="cuda").contiguous(memory_format=torch.channels_last)
        dst = big[:, :, 1::2, 0::2]
        ref = src
    elif case == "zero":
        dst = torch.ones(2, 8, 5, 6, device="cuda").contiguous(memory_format=torch.channels_last)
        src = torch.empty(0, 0, 0, 0, device="cuda")
        ref = torch.zeros(2, 8, 5, 6, device="cuda")
    elif case == "transpose":
        src = torch.randn(3, 3, 16, 64, device="cuda", generator=g).permute(3, 2, 0, 1)
        dst = torch.empty(64, 16, 3, 3, device="cuda").contiguous(memory_format=torch.channels_last)
        ref = src
    elif case == "acc_rows":
        src = torch.randn(2, 8, 5, 6, device="cuda", generator=g).contiguous(
            memory_format=torch.channels_last)
        big = torch.randn(2, 8, 10, 12, device="cuda", generator=g).contiguous(
            memory_format=torch.channels_last)
        want = big.clone()
        want[:, :, 1::2, 0::2] += src
        C.copy4d(big[:, :, 1::2, 0::2], src, accumulate=True)
        torch.testing.assert_close(big, want)
        return
    elif case == "acc_generic":
        src = torch.randn(4, 3, 9, 7, device="cuda", generator=g)
        dst = torch.randn(4, 4, 9, 7, device="cuda", generator=g)
        want = dst.clone()
        want[:, :3] += src
        C.copy4d(dst, src, accumulate=True)
        torch.testing.assert_close(dst, want)
        return
    else:
        dst = torch.randn(2, 8, 5, 6, device="cuda", generator=g)
        want = dst.clone()
        C.copy4d(dst, torch.empty(0, 0, 0, 0, device="cuda"), accumulate=True)
        torch.testing.assert_close(dst, want)
        return
    C.copy4d(dst, src)
    torch.testing.assert_close(dst, ref)


def test_dgrad_w_accumulates_into_out():
    """conv_nhwc_dgrad_w(out=, beta=1): out = dgrad + out (split-K and direct tilings)."""
    from tutorial_torch_distributed_data_parallel_amd._native import native

    C = native()
    g = torch.Generator(device="cuda").manual_seed(1)
    for (B, Cin, H, Cout, R) in [(8, 64, 14, 256, 1), (2, 256, 7, 64, 1), (4, 32, 12, 32, 3)]:
        w = torch.randn(Cout, Cin, R, R, device="cuda", generator=g).contiguous(
            memory_format=torch.channels_last) * 0.1
        dy = torch.randn(B, Cout, H, H, device="cuda", generator=g).contiguous(
            memory_format=torch.channels_last)
        base = torch.randn(B, Cin, H, H, device="cuda", generator=g).contiguous(
            memory_format=torch.channels_last)
        fresh = C.conv_nhwc_dgrad_w(dy, w, [B, Cin, H, H], 1, 1, R // 2, R // 2)
        out = base.clone()
        r = C.conv_nhwc_dgrad_w(dy, w, [B, Cin, H, H], 1, 1, R // 2, R // 2, out=out, beta=1.0)
        assert r.data_ptr() == out.data_ptr()
        torch.testing.assert_close(out, fresh + base, atol=1e-4, rtol=1e-4)


def test_padded_channels_last_input_and_native_flatten():
    """data/synthetic.py padded_channels_last: the stem conv reads the zero-padded NHWC storage
    in place (forward and weight gradient equal the plain NCHW input's); ops.flatten of a
    channels_last activation equals torch.flatten (values and gradient)."""
    from tutorial_torch_distributed_data_parallel_amd import ops
    from tutorial_torch_distributed_data_parallel_amd.data.synthetic import (
        SyntheticDataset, gather_batch, padded_channels_last)

    torch.manual_seed(3)
    x = torch.randn(6, 3, 33, 31, device="cuda")
    xp = padded_channels_last(x)
    assert xp.shape == x.shape and torch.equal(xp, x)
    w1 = torch.randn(16, 3, 5, 5, device="cuda", requires_grad=True)
    w2 = w1.detach().clone().requires_grad_()
    y1 = ops.conv2d(x, w1, None, 2, 2)
    y2 = ops.conv2d(xp, w2, None, 2, 2)
    torch.testing.assert_close(y1, y2)
    g = torch.randn_like(y1)
    y1.backward(g)
    y2.backward(g)
    torch.testing.assert_close(w1.grad, w2.grad)
    ds = SyntheticDataset(10, (3, 16, 16), device="cuda", seed=1)
    assert getattr(ds.x, "_tdp_padded_base", None) is not None
    idx = torch.tensor([3, 1, 7], device="cuda")
    xb, yb = gather_batch(ds.x, ds.y, idx)
    torch.testing.assert_close(xb, ds.x[idx.cpu()])
    assert torch.equal(yb, ds.y[idx])
    a = torch.randn(4, 8, 6, 6, device="cuda").contiguous(memory_format=torch.channels_last)
    a1 = a.clone().requires_grad_()
    a2 = a.clone().requires_grad_()
    f1 = ops.flatten(a1)
    f2 = torch.flatten(a2, 1)
    torch.testing.assert_close(f1, f2)
    gg = torch.randn_like(f1)
    f1.backward(gg)
    f2.backward(gg)
    torch.testing.assert_close(a1.grad, a2.grad)
    assert a1.grad.is_contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("shape", [(8, 64, 28, 28, 64, 3, 1), (4, 256, 14, 14, 1024, 1, 1),
                                   (2, 4, 33, 29, 64, 7, 2), (3, 128, 9, 9, 512, 1, 1),
                                   # 113 row tiles: two chunks of the partial merge (64 + 49)
                                   (16, 64, 30, 30, 64, 3, 1)])
def test_conv_epilogue_bn_stats(shape):
    """The forward GEMM epilogue's per-tile (count, mean, M2) merged by bn_moments_partials equal
    the moments pass over the stored output; ops.conv2d(bn_stats=True) -> batch_norm uses them."""
    from tutorial_torch_distributed_data_parallel_amd import ops
    from tutorial_torch_distributed_data_parallel_amd._native import native

    C = native()
    B, Cin, H, W, Cout, R, st = shape
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn(B, Cin, H, W, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last) + 0.7
    w = (torch.randn(Cout, Cin, R, R, device="cuda", generator=g) * 0.2).contiguous(
        memory_format=torch.channels_last)
    C.gemm_f32_set_override(0, 1, 0)  # unsplit: small test shapes would plan split-K
    try:
        y = ops.conv2d(x, w, None, st, R // 2, bn_stats=True)
    finally:
        C.gemm_f32_set_override(0, 0, 0)
    tag = getattr(y, "_tdp_bn_part", None)
    assert tag is not None, "an unsplit forward plan must emit statistics"
    rows = y.permute(0, 2, 3, 1).reshape(-1, Cout)
    ref = C.bn_moments(rows)[0]
    got = C.bn_moments_partials(tag[0], float(rows.shape[0]))
    torch.testing.assert_close(got[:Cout], ref[:Cout], atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(got[Cout:2 * Cout], ref[Cout:2 * Cout], atol=1e-5, rtol=1e-4)
    assert got[2 * Cout].item() == rows.shape[0]
    yd = y.double()
    torch.testing.assert_close(got[:Cout].double(), yd.mean((0, 2, 3)), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(got[Cout:2 * Cout].double(), yd.var((0, 2, 3), unbiased=False),
                               atol=1e-5, rtol=1e-4)
    # the batch norm consumes them: same output as when the moments pass runs
    gamma, beta = torch.randn(Cout, device="cuda"), torch.randn(Cout, device="cuda")
    o1 = ops.batch_norm(y, None, None, gamma, beta, training=True, relu=True)
    o2 = ops.batch_norm(y.clone(), None, None, gamma, beta, training=True, relu=True)
    torch.testing.assert_close(o1, o2, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("opt_name", ["sgd", "adam"])
def test_optimizer_on_channels_last_conv_weights_without_ddp(opt_name):
    """The native convolutions keep their weights channels_last; the multi-tensor optimizer path
    (no DDP arena) updates them in storage order, grads in either layout, like torch.optim."""
    import tutorial_torch_distributed_data_parallel_amd as tdp

    torch.manual_seed(0)
    w = torch.randn(8, 4, 3, 3, device="cuda").contiguous(memory_format=torch.channels_last)
    b = torch.randn(8, device="cuda")
    p1 = [torch.nn.Parameter(w.clone(memory_format=torch.channels_last)),
          torch.nn.Parameter(b.clone())]
    p2 = [torch.nn.Parameter(w.clone()), torch.nn.Parameter(b.clone())]
    o1 = (tdp.optim.SGD(p1, lr=0.1, momentum=0.9) if opt_name == "sgd"
          else tdp.optim.Adam(p1, lr=1e-2))
    o2 = (torch.optim.SGD(p2, lr=0.1, momentum=0.9) if opt_name == "sgd"
          else torch.optim.Adam(p2, lr=1e-2))
    for i in range(3):
        gw = torch.randn(8, 4, 3, 3, device="cuda")
        gb = torch.randn(8, device="cuda")
        # alternate the gradient layout: channels_last and plain contiguous
        p1[0].grad = gw.contiguous(memory_format=torch.channels_last) if i % 2 else gw.clone()
        p1[1].grad = gb.clone()
        p2[0].grad, p2[1].grad = gw.clone(), gb.clone()
        o1.step()
        o2.step()
    assert p1[0].is_contiguous(memory_format=torch.channels_last)
    for a, r in zip(p1, p2):
        torch.testing.assert_close(a.detach(), r.detach(), rtol=1e-5, atol=1e-6)
