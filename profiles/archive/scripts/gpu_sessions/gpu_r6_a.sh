#!/bin/bash
# Planes-A skinny GEMM: numerics tests, then the microbenchmark against the fast GEMM.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gemm_planes_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r6a_pytest.log 2>&1
rc=$?; tail -15 gpurun_out/r6a_pytest.log; fatal $rc pytest
timeout -k 10 200 python -u scripts/bench_gemm_planes.py > gpurun_out/r6a_bench.log 2>&1; rc=$?; cat gpurun_out/r6a_bench.log; fatal $rc bench
echo done
