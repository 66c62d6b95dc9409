#!/bin/bash
# Two-waves-per-SIMD planes GEMM (gemm_planes_set_cfg stages 4): numerics, driver-shaped bench
# A/B against the default 3-stage kernel (interleaved), and the dp1 kernel table under it.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9k; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gemm_planes_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r9k/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r9k/pytest.log; fatal $rc pytest
ms() { python3 -c 'import json,sys; print(json.load(open(sys.argv[1]))["ms_per_step"])' "$1"; }
for i in 1 2 3; do
for c in 3 4; do
timeout -k 10 300 python scripts/archive/run_with_variant.py --planes $c,0,0 -- bench.py --steps 20 --warmup 5 --no-diag > gpurun_out/r9k/c${c}_$i.json 2>gpurun_out/r9k/c${c}_$i.err; fatal $? c$c
echo "cfg $c run $i $(ms gpurun_out/r9k/c${c}_$i.json)"
done
done
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r9k/kt4 -o kt -- python3 scripts/archive/run_with_variant.py --planes 4,0,0 -- bench.py --steps 60 --warmup 10 --no-diag > gpurun_out/r9k/kt4.log 2>&1; fatal $? kt4
T=$(find gpurun_out/r9k/kt4 -name '*kernel_trace.csv' | head -1)
python3 scripts/step_kernels.py $T ce_fwd 40 > gpurun_out/r9k/dp1_kernels_c4.md
cat gpurun_out/r9k/dp1_kernels_c4.md
echo done
