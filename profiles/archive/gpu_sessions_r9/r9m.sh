#!/bin/bash
# Tensor-sharded step: GPU tests (peer vehicle), per-rank compute proxy at W = 1/2/4/8.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9m; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_tensor_parallel_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r9m/pytest.log 2>&1; rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r9m/pytest.log | tail -12; fatal $rc pytest
timeout -k 10 300 python -u scripts/tp_rank_proxy.py > gpurun_out/r9m/proxy.jsonl 2> gpurun_out/r9m/proxy.err; rc=$?; cat gpurun_out/r9m/proxy.jsonl; tail -3 gpurun_out/r9m/proxy.err; fatal $rc proxy
echo done
