#!/bin/bash
# fused bias+act / folded 1/W: TP GPU tests, kernels tests, proxy, W=8 kernel table.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9x; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 700 python -u -m pytest tests/test_tensor_parallel_gpu.py tests/test_kernels_gpu.py tests/test_ddp_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r9x/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r9x/pytest.log; grep FAIL gpurun_out/r9x/pytest.log | head -3; fatal $rc pytest
timeout -k 10 300 python -u scripts/tp_rank_proxy.py > gpurun_out/r9x/proxy.jsonl 2> gpurun_out/r9x/proxy.err; rc=$?; grep W gpurun_out/r9x/proxy.jsonl; fatal $rc proxy
echo done
