#!/bin/bash
# The tensor-sharded GPU tests after the accumulation fix (early replicated all-reduce joined).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9am; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 500 python -u -m pytest tests/test_tensor_parallel_gpu.py -x -v --timeout 180 --timeout-method thread > gpurun_out/r9am/tp_tests.log 2>&1; rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed|Mismatch|Greatest" gpurun_out/r9am/tp_tests.log | tail -22; fatal $rc tp_tests
echo done
