#!/bin/bash
# Tensor-sharded step with the shards' SGD in their weight-gradient GEMM epilogues: parity tests,
# per-rank proxy fused vs unfused at W = 2 / 4 / 8, kernel trace at W = 2.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9ak; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 500 python -u -m pytest tests/test_tensor_parallel_gpu.py -x -v --timeout 180 --timeout-method thread > gpurun_out/r9ak/tp_tests.log 2>&1; rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r9ak/tp_tests.log | tail -20; fatal $rc tp_tests
timeout -k 10 300 python -u scripts/tp_rank_proxy.py 2 4 8 > gpurun_out/r9ak/proxy_fused.jsonl 2> gpurun_out/r9ak/proxy_fused.err; rc=$?; cat gpurun_out/r9ak/proxy_fused.jsonl; fatal $rc proxy_fused
timeout -k 10 300 python -u scripts/tp_rank_proxy.py --no-dp1 --unfused 2 4 8 > gpurun_out/r9ak/proxy_unfused.jsonl 2> gpurun_out/r9ak/proxy_unfused.err; rc=$?; cat gpurun_out/r9ak/proxy_unfused.jsonl; fatal $rc proxy_unfused
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r9ak/kt2 -o kt -- python3 scripts/tp_rank_proxy.py --no-dp1 2 > gpurun_out/r9ak/kt2.log 2>&1; fatal $? kt2
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r9ak/kt8 -o kt -- python3 scripts/tp_rank_proxy.py --no-dp1 8 > gpurun_out/r9ak/kt8.log 2>&1; fatal $? kt8
echo done
