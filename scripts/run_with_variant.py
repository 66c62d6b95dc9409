"""Run a script (bench.py by default) with native measurement settings applied first, in the
same process -- the A/B switches are setters, not environment knobs (README "Environment
knobs"). Example (optimizer-epilogue variant 28 = LDS + non-temporal + one batch per tile):

    python scripts/run_with_variant.py --sgd 28 -- bench.py --steps 100
"""
import argparse
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sgd", type=int, default=-1, help="SGD epilogue variant flags")
    ap.add_argument("--adam", type=int, default=-1, help="Adam epilogue variant flags")
    ap.add_argument("--persist", type=int, default=-1)
    ap.add_argument("--wgs", type=int, default=-1)
    ap.add_argument("--planes", type=str, default=None, help="stages,pf,splits")
    ap.add_argument("--no-early-g", action="store_true",
                    help="factored g gathers only from the layer's own backward")
    ap.add_argument("--no-pair-wgrad", action="store_true",
                    help="world size 1: one launch per weight-gradient + optimizer GEMM")
    ap.add_argument("--no-local1d", action="store_true",
                    help="one-rank BatchNorm1d through the split kernels (statistics, then "
                         "normalisation; sums, then input gradient)")
    ap.add_argument("--no-bn-update", action="store_true",
                    help="one-launch BatchNorm1d backward without the in-place optimizer step "
                         "on w / b (the reducer's flat pass updates them)")
    ap.add_argument("--no-sync1d", action="store_true",
                    help="SyncBatchNorm over a batch of rows through the split kernels")
    ap.add_argument("rest", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    rest = a.rest[1:] if a.rest[:1] == ["--"] else a.rest
    script = rest[0] if rest else os.path.join(ROOT, "bench.py")
    from tutorial_torch_distributed_data_parallel_amd._native import native

    C = native()
    C.gemm_f32_set_opt_variant(sgd=a.sgd, adam=a.adam, persist=a.persist, wgs=a.wgs)
    if a.planes:
        st, pf, sp = (int(v) for v in a.planes.split(","))
        if not C.gemm_planes_set_cfg(st, pf, sp):
            raise SystemExit(f"invalid planes config {a.planes}")
    if a.no_early_g:
        import importlib

        importlib.import_module("tutorial_torch_distributed_data_parallel_amd.ops.linear") \
            .set_early_prev_g(False)
    if a.no_pair_wgrad:
        import importlib

        importlib.import_module("tutorial_torch_distributed_data_parallel_amd.ops.linear") \
            .set_pair_wgrad(False)
    if a.no_local1d:
        import importlib

        importlib.import_module("tutorial_torch_distributed_data_parallel_amd.ops.norm") \
            .set_local1d(False)
    if a.no_bn_update:
        import importlib

        importlib.import_module("tutorial_torch_distributed_data_parallel_amd.ops.norm") \
            .set_local1d(True, update=False)
    if a.no_sync1d:
        import importlib

        importlib.import_module("tutorial_torch_distributed_data_parallel_amd.ops.norm") \
            .set_sync1d(False)
    sys.argv = [script] + rest[1:]
    runpy.run_path(script if os.path.isabs(script) else os.path.join(ROOT, script),
                   run_name="__main__")


if __name__ == "__main__":
    main()
