"""Large-tile split-bf16 GEMM (csrc/gemm_emu8.hip: 256 x 256 tile, 8 waves, one workgroup per
CU) against the fast kernel (gemm_f32_fast.hip, split-bf16 products) on square and
convolution-like shapes, interleaved in one process. One JSON line per shape: microseconds,
TFLOP/s of each, and whether the two results are bitwise equal (same products, same k order).

python scripts/bench_gemm_emu8.py"""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from tutorial_torch_distributed_data_parallel_amd._native import native  # noqa: E402

C = native()
dev = "cuda"
SHAPES = [("sq4096_nt", 4096, 4096, 4096, True), ("sq4096_nn", 4096, 4096, 4096, False),
          ("sq8192_nt", 8192, 8192, 8192, True),
          ("r50_3x3_l1", 401408, 64, 576, True), ("r50_1x1_l1", 401408, 256, 64, True),
          ("r50_3x3_l3", 25088, 256, 2304, True), ("r50_1x1_l3", 25088, 1024, 256, True),
          ("rep_fc1", 4096, 9216, 1024, False), ("alex_fc", 4096, 4096, 9216, True)]


def timeit(fn, reps):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps * 1000.0


x = torch.randn(4096, 4096, device=dev)
for _ in range(40):
    torch.mm(x, x)
torch.cuda.synchronize()

for name, M, N, K, bk in SHAPES:
    torch.manual_seed(M + N + K)
    A = torch.randn(M, K, device=dev)
    B = torch.randn((N, K) if bk else (K, N), device=dev)
    o8 = torch.empty(M, N, device=dev)
    of = torch.empty(M, N, device=dev)
    fl = 2.0 * M * N * K
    reps = 5 if fl > 4e12 else 20
    o4 = torch.empty(M, N, device=dev)
    best = {}
    for _ in range(3):
        for w, o in ((8, o8), (4, o4)):
            C.gemm_emu8_set_waves(w)
            best[f"w{w}"] = min(best.get(f"w{w}", 1e30),
                                timeit(lambda: C.gemm_emu8(A, B, o, bk), reps))
        C.gemm_f32_set_mode(2)  # the 128 x 128 fast kernel (auto dispatch may pick emu8)
        best["fast"] = min(best.get("fast", 1e30),
                           timeit(lambda: C.gemm_f32(A, B, of, True, bk), reps))
        C.gemm_f32_set_mode(0)
    C.gemm_emu8_set_waves(8)
    torch.cuda.synchronize()
    Bm = B.t() if bk else B
    rows = torch.randperm(M, device=dev)[:256]
    ref = A[rows].double() @ Bm.double()
    scale = A[rows].double().abs() @ Bm.double().abs()
    err = ((o8[rows].double() - ref).abs() / scale.clamp_min(1e-30)).max().item()
    row = {"shape": [M, N, K, bk], "w8_equal": bool(torch.equal(o8, of)), "w4_equal": bool(torch.equal(o4, of)),
           "err8_over_u": round(err / 2.0 ** -24, 2)}
    for k, us in best.items():
        row[k + "_us"] = round(us, 1)
        row[k + "_tflops"] = round(fl / us / 1e6, 1)
    row["speedup_w8"] = round(best["fast"] / best["w8"], 3)
    row["speedup_w4"] = round(best["fast"] / best["w4"], 3)
    print(json.dumps({name: row}), flush=True)
