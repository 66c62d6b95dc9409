#!/bin/bash
# Weight-gradient epilogue GEMM plan variants under the fused tensor-sharded per-rank step.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9ap; export TMPDIR=/tmp
timeout -k 10 400 python -u dev/micro/tp_wgrad_variants.py 2 8 > gpurun_out/r9ap/variants.jsonl 2> gpurun_out/r9ap/variants.err; rc=$?; cat gpurun_out/r9ap/variants.jsonl; tail -3 gpurun_out/r9ap/variants.err; exit $rc
