"""fp32 GEMM from pre-split bf16 planes (csrc/gemm_planes.hip): the split is exact (three RNE
bf16 planes sum back to every fp32 value, K padding zero) and the planes GEMM carries fp32
accuracy against fp64, like the in-kernel split path (tests/test_gemm_emu_gpu.py) and the native
v_mfma_f32_32x32x2_f32 path."""
import pytest
import torch

pytestmark = pytest.mark.gpu

U = 2.0 ** -24


@pytest.fixture(scope="module")
def C():
    from tutorial_torch_distributed_data_parallel_amd._native import native

    return native()


@pytest.mark.parametrize("kcontig", [True, False])
@pytest.mark.parametrize("R,K", [(64, 32), (130, 77), (300, 1000)])
def test_split_planes_exact(C, kcontig, R, K):
    torch.manual_seed(R + K)
    x = torch.randn(R, K, device="cuda") * torch.exp2(torch.randint(-30, 31, (R, K),
                                                                    device="cuda").float())
    src = x if kcontig else x.t().contiguous()
    planes = C.split_planes(src, kcontig)
    Kp = (K + 31) // 32 * 32
    assert planes.shape == (3, R, Kp) and planes.dtype == torch.bfloat16
    back = planes.double().sum(0)
    assert torch.equal(back[:, :K], x.double())
    assert torch.count_nonzero(back[:, K:]) == 0
    # RNE head term: the first plane is the bf16 rounding of x
    assert torch.equal(planes[0, :, :K], x.bfloat16())


def _err(out, A2, B2):
    ref = A2 @ B2
    scale = A2.abs() @ B2.abs()
    return ((out.double() - ref).abs() / scale.clamp_min(1e-30)).max().item()


SHAPES = [(256, 128, 32, True, True), (300, 200, 100, True, True), (130, 66, 257, False, True),
          (512, 384, 640, True, False), (1000, 520, 96, False, False),
          (2048, 2048, 512, True, True)]


@pytest.mark.parametrize("M,N,K,ak,bk", SHAPES)
@pytest.mark.parametrize("dist", ["normal", "wide"])
def test_planes_gemm_fp32_accuracy(C, M, N, K, ak, bk, dist):
    torch.manual_seed(M + 3 * N + 7 * K)
    A = torch.randn((M, K) if ak else (K, M), device="cuda")
    B = torch.randn((N, K) if bk else (K, N), device="cuda")
    if dist == "wide":
        A = A * torch.exp2(torch.randint(-20, 21, A.shape, device="cuda").float())
        B = B * torch.exp2(torch.randint(-20, 21, B.shape, device="cuda").float())
    out = torch.empty(M, N, device="cuda")
    C.gemm_f32_planes(A, B, out, ak, bk)
    nat = torch.empty(M, N, device="cuda")
    C.gemm_f32_set_emu(False)
    try:
        C.gemm_f32(A, B, nat, ak, bk)
    finally:
        C.gemm_f32_set_emu(True)
    torch.cuda.synchronize()
    A2 = (A if ak else A.t()).double()
    B2 = (B.t() if bk else B).double()
    e, e_nat = _err(out, A2, B2), _err(nat, A2, B2)
    bound = (8 + 2 * K ** 0.5) * U
    assert e < bound, (e, e_nat, bound)
    assert e < 4 * e_nat + 16 * U, (e, e_nat)


def test_planes_gemm_epilogue(C):
    torch.manual_seed(2)
    x = torch.randn(300, 320, device="cuda")
    w = torch.randn(200, 320, device="cuda") / 18
    b = torch.randn(200, device="cuda")
    out = torch.randn(300, 200, device="cuda")
    prev = out.clone()
    C.gemm_f32_planes(x, w, out, True, True, bias=b, beta=0.5, relu=True)
    ref = torch.relu(x.double() @ w.double().t() + b.double() + 0.5 * prev.double()).float()
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
