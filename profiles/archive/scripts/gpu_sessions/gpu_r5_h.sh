#!/bin/bash
# Pre-split planes GEMM: numerics, then speed vs the in-kernel split GEMM.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm_planes_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5h_pytest.log 2>&1; rc=$?
tail -15 gpurun_out/r5h_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_gemm_planes.py > gpurun_out/r5h_bench.jsonl 2> gpurun_out/r5h_bench.err; rc=$?
cat gpurun_out/r5h_bench.jsonl; tail -3 gpurun_out/r5h_bench.err; exit $rc
