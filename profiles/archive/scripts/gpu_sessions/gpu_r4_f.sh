#!/bin/bash
# Toy-MLP GEMM plan sweep (tile width / split-K / stages) under split-bf16 products.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/bench_gemm.py > gpurun_out/r4f_gemm_sweep.log 2>&1
rc=$?; cut -c1-1200 gpurun_out/r4f_gemm_sweep.log; exit $rc
