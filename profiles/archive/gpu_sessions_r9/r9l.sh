#!/bin/bash
# Large-tile split-bf16 GEMM (gemm_emu8) vs the fast kernel: rates, bitwise agreement, fp64 error.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9l; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/bench_gemm_emu8.py > gpurun_out/r9l/emu8.jsonl 2> gpurun_out/r9l/emu8.err; rc=$?
grep -v amdgpu.ids gpurun_out/r9l/emu8.jsonl; tail -5 gpurun_out/r9l/emu8.err; exit $rc
