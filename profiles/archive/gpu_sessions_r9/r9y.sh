#!/bin/bash
# gemm_f32 auto-dispatch to the 256x256 kernel: tests, GEMM bench, dp1 sanity.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9y; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gemm_emu_gpu.py tests/test_tensor_parallel_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r9y/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r9y/pytest.log; grep FAIL gpurun_out/r9y/pytest.log | head; fatal $rc pytest
timeout -k 10 300 python -u scripts/bench_gemm_emu8.py > gpurun_out/r9y/emu8.jsonl 2>/dev/null; fatal $? emu8; head -3 gpurun_out/r9y/emu8.jsonl | cut -c1-220
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-diag > gpurun_out/r9y/d.json 2>/dev/null; fatal $? bench; python3 -c 'import json; print(json.load(open("gpurun_out/r9y/d.json"))["ms_per_step"])'
echo done
