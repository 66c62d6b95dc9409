#!/bin/bash
# Optimizer-epilogue GEMM: tile width x pipeline depth x persistent workgroups per CU (micro-benchmark).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r23; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 150 python scripts/bench_opt_epilogue.py > $O/epi.jsonl 2> $O/epi.err
rc=$?
cat $O/epi.jsonl
exit $rc
