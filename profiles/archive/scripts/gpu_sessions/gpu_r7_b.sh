#!/bin/bash
# Split-K fix-up in the planes GEMM (no planes_reduce_kernel), sliced cursor gather, grouped
# factor all-gathers:
# targeted GPU tests, interleaved A/B of the toy-MLP step, kernel table.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r7b; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 900 python -u -m pytest tests/test_gemm_planes_gpu.py tests/test_factor_gpu.py tests/test_ddp_gpu.py tests/test_sync_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r7b/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r7b/pytest.log; fatal $rc pytest
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["config"].get("final_loss"))' $1; }
for r in 1 2 3; do
timeout -k 10 300 python bench.py --no-diag > gpurun_out/r7b/b.json 2>/dev/null; fatal $? b; echo "fixup r$r $(ms gpurun_out/r7b/b.json)"
TDP_PLANES_FIXUP=0 timeout -k 10 300 python bench.py --no-diag > gpurun_out/r7b/b0.json 2>/dev/null; fatal $? b0; echo "reduce r$r $(ms gpurun_out/r7b/b0.json)"
TDP_CURSOR_ROWS=0 timeout -k 10 300 python bench.py --no-diag > gpurun_out/r7b/b1.json 2>/dev/null; fatal $? b1; echo "fixup, 1-wg-per-row gather r$r $(ms gpurun_out/r7b/b1.json)"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-diag > gpurun_out/r7b/d.json 2>/dev/null; fatal $? d; echo "driver-shaped $(ms gpurun_out/r7b/d.json)"
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r7b/prof -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r7b/prof.log 2>&1; fatal $? prof
python3 scripts/step_kernels.py $(find gpurun_out/r7b/prof -name '*kernel_trace.csv' | head -1) ce_fwd 40 > gpurun_out/r7b/mlp_kernels.md
cat gpurun_out/r7b/mlp_kernels.md
python3 scripts/step_timeline.py $(find gpurun_out/r7b/prof -name '*kernel_trace.csv' | head -1) ce_fwd 40 > gpurun_out/r7b/mlp_timeline.md
cat gpurun_out/r7b/mlp_timeline.md
echo done
