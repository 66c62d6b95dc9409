#!/bin/bash
# Stage-unrolled, explicitly interleaved 3-stage planes GEMM: numerics, kernel times, step time.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r6r; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gemm_planes_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6r/pytest.log 2>&1
rc=$?; tail -1 gpurun_out/r6r/pytest.log; fatal $rc pytest
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6r/kt -o kt -- python3 scripts/planes_pmc_probe.py > gpurun_out/r6r/kt.log 2>&1; fatal $? kt
ms() { python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["config"].get("final_loss"))' $1; }
for r in 1 2; do
timeout -k 10 300 python bench.py --no-diag > gpurun_out/r6r/b.json 2>/dev/null; fatal $? b; echo "default r$r $(ms gpurun_out/r6r/b.json)"
done
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6r/prof -o kt -- python3 bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r6r/prof.log 2>&1; fatal $? prof
python3 scripts/step_kernels.py $(find gpurun_out/r6r/prof -name '*kernel_trace.csv' | head -1) ce_fwd 40 > gpurun_out/r6r/mlp_kernels.md
head -8 gpurun_out/r6r/mlp_kernels.md
echo done
