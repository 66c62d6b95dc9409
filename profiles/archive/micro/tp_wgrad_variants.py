"""Per-rank tensor-sharded step (fused shard update) under weight-gradient epilogue GEMM plan
variants: persistent workgroups per CU, non-persistent grid, 128 x 64 tiles (global overrides,
a measurement only). One JSON line per (W, variant)."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/dev/", 1)[0])
import tutorial_torch_distributed_data_parallel_amd as tdp  # noqa: E402
from tutorial_torch_distributed_data_parallel_amd._native import native  # noqa: E402
from tutorial_torch_distributed_data_parallel_amd.parallel.tensor_parallel import \
    rank_compute_ms  # noqa: E402

tdp.init_process_group("nccl", rank=0, world_size=1, local_rank=0)
C = native()
a = torch.randn(4096, 4096, device="cuda")
for _ in range(50):
    a @ a
torch.cuda.synchronize()
VARIANTS = {
    "default": lambda: None,
    "wgs3": lambda: C.gemm_f32_set_opt_variant(wgs=3),
    "wgs1": lambda: C.gemm_f32_set_opt_variant(wgs=1),
    "nonpersist": lambda: C.gemm_f32_set_opt_variant(persist=0),
}
for W in [int(v) for v in sys.argv[1:]] or [2, 8]:
    for name, setv in VARIANTS.items():
        setv()
        try:
            ms = rank_compute_ms(W, steps=200)
        finally:
            C.gemm_f32_set_opt_variant(wgs=2, persist=1)
        print(json.dumps({"W": W, "variant": name, "rank_compute_ms": round(ms, 4)}), flush=True)
